"""GPU parity of the fused MLP kernels (forward / losses / policy gradient / Fisher
product / VF loss-grad) against the float64 oracle, through the C ABI."""
import numpy as np
import pytest
import torch

from oracle import trpo_np as T

pytestmark = pytest.mark.gpu

CASES = [("gauss", 11, 3), ("softmax", 4, 2), ("gauss", 17, 6), ("softmax", 6, 5)]


def _net(head, nin, nout):
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    h = {"gauss": _lib.HEAD_GAUSS, "softmax": _lib.HEAD_SOFTMAX, "linear": _lib.HEAD_LINEAR}[head]
    return MlpNet(nin, nout, h)


def _setup(head, nin, nout, N, seed=0):
    rng = np.random.default_rng(seed)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldth = th + 0.01 * rng.standard_normal(spec.P)
    oldprob = T.policy_prob(spec, oldth, ob).astype(np.float32).astype(np.float64)
    noise = rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N)
    act = T.sample(spec, oldprob, noise)
    if head == "gauss":
        act = act.astype(np.float32).astype(np.float64)
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    return spec, th, ob, act, adv, oldprob


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("head,nin,nout", CASES)
@pytest.mark.parametrize("N", [1, 77, 1000])
def test_forward_prob(head, nin, nout, N):
    spec, th, ob, *_ = _setup(head, nin, nout, N)
    net = _net(head, nin, nout)
    net.set_flat(th)
    got = net.forward(_dev(ob), N).cpu().numpy().astype(np.float64)
    want = T.policy_prob(spec, th, ob)
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("head,nin,nout", CASES)
def test_losses_and_policy_gradient(head, nin, nout):
    from modular_rl_amd import _lib
    N = 2000
    spec, th, ob, act, adv, oldprob = _setup(head, nin, nout, N, seed=1)
    net = _net(head, nin, nout)
    net.set_flat(th)
    x = _dev(ob)
    a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
             ghead=ghead, partial=partial)
    sums = torch.zeros(4, dtype=torch.float64, device="cuda")
    net.reduce_partial(partial, N, sums)
    g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, g)
    s = sums.cpu().numpy()
    losses = np.array([-s[0] / N, s[1] / N, s[2] / N])
    want = T.surr_kl_ent(spec, th, ob, act, adv, oldprob)
    np.testing.assert_allclose(losses, want, rtol=1e-4, atol=1e-6)
    gw = T.policy_gradient(spec, th, ob, act, adv, oldprob)
    assert _rel(g.cpu().numpy(), gw) < 1e-4


@pytest.mark.parametrize("head,nin,nout", CASES)
def test_fisher_vector_product(head, nin, nout):
    from modular_rl_amd import _lib
    N = 3000
    spec, th, ob, *_ = _setup(head, nin, nout, N, seed=2)
    rng = np.random.default_rng(5)
    v = rng.standard_normal(spec.P).astype(np.float32)
    net = _net(head, nin, nout)
    net.set_flat(th)
    x = _dev(ob)
    vt = _dev(v)
    imgt = torch.zeros_like(net.image)
    net.pack(theta=vt, image=imgt, fwd_only=True)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt, image_t=imgt)
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, fv)
    want = T.fisher_vector_product(spec, th, v.astype(np.float64), ob)
    assert _rel(fv.cpu().numpy(), want) < 1e-4


@pytest.mark.parametrize("nin,cus", [(5, 0), (12, 0), (12, 1), (12, 5)])
def test_value_forward_and_loss_grad_with_time_feature(nin, cus):
    """cus > 0: the passes sized for a CU subset (the VF fit beside the rollout); at
    N = 1500 (12 blocks) cus 1 caps the VJP at 1 block and the row passes at 6, cus 5
    the VJP at 5 -- the partial / slab rows follow and the sums stay exact."""
    from modular_rl_amd import _lib
    N, limit = 1500, 200.0
    rng = np.random.default_rng(3)
    spec = T.Spec(nin, [64, 64], 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.05 * rng.standard_normal(spec.P)).astype(np.float32).astype(np.float64)
    obs = rng.standard_normal((N, nin - 1)).astype(np.float32)
    ept = rng.integers(0, 200, size=N).astype(np.int32)
    X = np.concatenate([obs.astype(np.float64), (ept / limit).astype(np.float32).astype(np.float64)[:, None]], axis=1)
    y = rng.standard_normal(N).astype(np.float32)
    net = _net("linear", nin, 1)
    net.size_for_cus(cus)
    net.set_flat(th)
    xo, et = _dev(obs), _dev(ept, torch.int32)
    if cus:
        assert net.partial_rows(N) == 4 * min(12, 6 * cus)
    v = net.forward(xo, N, ep_t=et, timestep_limit=limit).cpu().numpy()
    want_v = T.mlp_forward(spec, th, X)[0][:, 0]
    np.testing.assert_allclose(v, want_v, rtol=2e-5, atol=2e-6)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    ghead = torch.zeros(N, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_VFLOSS, xo, N, ep_t=et, timestep_limit=limit, inv_n_global=1.0 / N, target=_dev(y),
             ghead=ghead, partial=partial)
    sums = torch.zeros(4, dtype=torch.float64, device="cuda")
    net.reduce_partial(partial, N, sums)
    g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(xo, N, ghead, g, ep_t=et, timestep_limit=limit)
    loss, gw, mse, l2 = T.vf_loss_grad(spec, th, X, y.astype(np.float64))
    np.testing.assert_allclose(sums[0].item() / N, mse, rtol=1e-5)
    assert _rel(g.cpu().numpy() + 2e-3 * th, gw) < 1e-4


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2)])
def test_activation_cache_is_bitwise_transparent(head, nin, nout, monkeypatch):
    """SURRGRAD stores h1/h2; the FVP rows pass that follows reads them instead of
    recomputing the forward -- its head rows must equal the uncached kernel's bit for bit
    (the exact-f32 row kernels: MRL_ROWS_SPLIT=0; the split forward's cache holds its own
    rounding, tests/test_gpu_split.py).
    The cached VJP is the transpose-free 16-row kernel (mlp_vjp16_kernel): the same sums
    in another row order, so its gradients agree with the uncached 32-row kernel to fp32
    rounding and both with the float64 oracle."""
    from modular_rl_amd import _lib
    monkeypatch.setenv("MRL_ROWS_SPLIT", "0")
    N = 3000
    spec, th, ob, act, adv, oldprob = _setup(head, nin, nout, N, seed=9)
    v = np.random.default_rng(2).standard_normal(spec.P).astype(np.float32)
    outs = []
    for use_cache in (False, True):
        net = _net(head, nin, nout)
        net.use_cache = use_cache
        net.set_flat(th)
        x, vt = _dev(ob), _dev(v)
        a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
        partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
        g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
                 ghead=ghead, partial=partial)
        net.vjp_flat(x, N, ghead, g)
        imgt = torch.zeros_like(net.image)
        net.pack(theta=vt, image=imgt, fwd_only=True)
        fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt, image_t=imgt)
        gh = ghead.clone()
        net.vjp_flat(x, N, ghead, fv)
        outs.append((g.cpu(), gh.cpu(), fv.cpu()))
        if use_cache:
            assert net._cache_key is not None
    (g_u, gh_u, fv_u), (g_c, gh_c, fv_c) = outs
    assert torch.equal(gh_u, gh_c)
    assert _rel(g_c.numpy(), g_u.numpy()) < 1e-5
    assert _rel(fv_c.numpy(), fv_u.numpy()) < 1e-5
    want = T.fisher_vector_product(spec, th, v.astype(np.float64), ob)
    for fv in (fv_u, fv_c):
        assert _rel(fv.numpy(), want) < 1e-4
    gw = T.policy_gradient(spec, th, ob, act, adv, oldprob)
    for g in (g_u, g_c):
        assert _rel(g.numpy(), gw) < 1e-4


@pytest.mark.parametrize("head,nin,nout", CASES)
@pytest.mark.parametrize("N", [1, 17, 3001])
def test_cached_fisher_product_and_gradient(head, nin, nout, N):
    """The cached VJP (16-row transpose-free kernel) after a recording SURRGRAD pass:
    policy gradient and Fisher product vs the float64 oracle on ragged row counts
    (partial 16- and 32-row tiles), wide inputs (nin 17: two gW0 tiles) and heads of
    more than four outputs (two head k-steps)."""
    from modular_rl_amd import _lib
    spec, th, ob, act, adv, oldprob = _setup(head, nin, nout, N, seed=11)
    v = np.random.default_rng(4).standard_normal(spec.P).astype(np.float32)
    net = _net(head, nin, nout)
    net.set_flat(th)
    x, vt = _dev(ob), _dev(v)
    a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
             ghead=ghead, partial=partial)
    assert net._cache_key is not None
    g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, g)
    assert _rel(g.cpu().numpy(), T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 1e-4
    imgt = torch.zeros_like(net.image)
    net.pack(theta=vt, image=imgt, fwd_only=True)
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt, image_t=imgt)
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, fv)
    assert _rel(fv.cpu().numpy(), T.fisher_vector_product(spec, th, v.astype(np.float64), ob)) < 1e-4
