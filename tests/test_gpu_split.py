"""The fp32 Fisher product on the bf16 matrix cores -- the split-operand JVP rows
(csrc/mlp_split.hip: fp32 operands split exactly into three bf16 parts, the part products
on bf16 MFMA with f32 accumulation) and the hybrid cached VJP (mlp_vjp16_kernel<HYB>: its
two 64x64 products on split operands) -- against the float64 oracle at north_star's 1e-4
and against the exact-f32 kernels to f32 rounding."""
import numpy as np
import pytest
import torch

from oracle import trpo_np as T

pytestmark = pytest.mark.gpu

CASES = [("gauss", 11, 3), ("softmax", 4, 2), ("gauss", 17, 6), ("softmax", 6, 5), ("gauss", 32, 8)]


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("head,nin,nout", CASES)
@pytest.mark.parametrize("N", [1, 33, 3001])
def test_split_fisher_product(head, nin, nout, N, monkeypatch):
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    rng = np.random.default_rng(nin * 7 + N)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    v = rng.standard_normal(spec.P).astype(np.float32)
    net = MlpNet(nin, nout, _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX)
    assert net.fisher_split
    net.set_flat(th)
    x, vt = _dev(ob), _dev(v)
    a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    gh = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob), ghead=gh,
             partial=partial)
    # exact-f32 kernel (f32 tangent image) and the split kernel (split tangent image)
    img32 = torch.zeros_like(net.image)
    net.pack(theta=vt, image=img32, fwd_only=True)
    gh32 = torch.zeros_like(gh)
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh32, tangent=vt, image_t=img32)
    imgs = net.new_tangent_image()
    net.pack_tangent(vt, imgs)
    ghs = torch.full_like(gh, float("nan"))
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghs, tangent=vt, image_t=imgs)
    a32, asp = gh32.cpu().numpy(), ghs.cpu().numpy()
    assert np.isfinite(asp).all()
    # the same rows to f32 rounding (different summation order of exact products)
    np.testing.assert_allclose(asp, a32, rtol=2e-5, atol=2e-6 * np.abs(a32).max())
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghs, fv)  # the hybrid cached VJP (policy net)
    want = T.fisher_vector_product(spec, th, v.astype(np.float64), ob)
    assert _rel(fv.cpu().numpy(), want) < 1e-4
    # the hybrid VJP against the exact-f32 VJP (the uncached kernel: an explicit image
    # bypasses the activation cache) on the same head rows: f32 rounding apart
    fs, f32 = torch.zeros_like(fv), torch.zeros_like(fv)
    net.vjp_flat(x, N, gh32, fs)
    net.vjp_flat(x, N, gh32, f32, image=net.image)
    assert _rel(fs.cpu().numpy(), f32.cpu().numpy()) < 1e-5
    assert _rel(f32.cpu().numpy(), want) < 1e-4


def test_split_image_parts_sum_to_the_f32_weights(monkeypatch):
    """The split image's three bf16 parts of every weight add up to the f32 weight
    exactly (the exact split the kernel's products rely on)."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    net = MlpNet(11, 3, _lib.HEAD_GAUSS)
    rng = np.random.default_rng(1)
    th = (rng.standard_normal(net.P) * np.exp(rng.uniform(-20, 5, net.P))).astype(np.float32)
    net.set_flat(th)
    img = net.image_s.cpu().numpy().view(np.uint32)
    fa0 = 64 + 64 + 2 * 8 * 32 + 16
    fwd_words = fa0 + 2 * 1 * 64 * 4 + 2 * 4 * 64 * 4
    FW = fwd_words - fa0
    assert img.size == fa0 + 3 * FW  # the forward section only (the VJP half splits its own operands)

    def bf(u):  # bf16 bits (low / high halves of the words) -> f32
        return (u.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    parts = [img[fa0 + p * FW: fa0 + (p + 1) * FW] for p in range(3)]
    for half in (0, 1):
        vals = [bf((pp >> (16 * half)) & 0xFFFF) for pp in parts]
        tot = vals[0] + vals[1] + vals[2]
        # every weight is an f32 value and the three parts reproduce it exactly
        assert np.array_equal(tot.astype(np.float32).astype(np.float64), tot)
        assert np.all(np.abs(vals[1]) <= np.abs(vals[0]) * 2.0 ** -7 + 1e-45)
    w32 = set(np.abs(th).astype(np.float64).tolist()) | {0.0}
    tot0 = np.abs(bf(img[fa0:fa0 + FW] & 0xFFFF) + bf(img[fa0 + FW:fa0 + 2 * FW] & 0xFFFF) +
                  bf(img[fa0 + 2 * FW:fa0 + 3 * FW] & 0xFFFF))
    assert set(tot0.tolist()) <= w32


def test_split_fisher_product_is_deterministic(monkeypatch):
    """The same split JVP-rows launch on the same 1 M rows gives the same bits every time
    (round 4's kernel did not: head_finish's ds_bpermute read packed-f32 head sums one
    instruction after their v_pk_add_f32 and returned stale values of lanes 48-63, a few
    16-row groups per 4 M rows; the cross-lane sums now use VALU permutes, DESIGN §3, and
    tools/isa_hazard_check.py guards the built code; the 4.19 M-row check is
    tests/test_gpu_fullsize.py)."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet, glorot_init
    N = 1 << 20
    rng = np.random.default_rng(0)
    net = MlpNet(11, 3, _lib.HEAD_GAUSS)
    net.set_flat(glorot_init(rng, 11, 3, _lib.HEAD_GAUSS))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, 11, device="cuda", generator=g)
    act = torch.randn(N, 3, device="cuda", generator=g)
    adv = torch.randn(N, device="cuda", generator=g)
    prob = net.forward(x, N).clone()
    gh = torch.zeros(N * net.gh, device="cuda")
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh, partial=partial)
    v = torch.randn(net.P, device="cuda", generator=g) * 1e-2
    imgt = net.new_tangent_image()
    net.pack_tangent(v, imgt)
    outs = []
    for _ in range(4):
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgt)
        outs.append(gh.clone())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    # and the hybrid cached VJP of those rows
    fv = [torch.zeros(net.P, device="cuda") for _ in range(3)]
    for f in fv:
        net.vjp_flat(x, N, gh, f)
    for f in fv[1:]:
        assert torch.equal(f, fv[0])


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2), ("linear", 12, 1), ("gauss", 17, 4)])
@pytest.mark.parametrize("N", [1, 33, 70001])
def test_vjp16_hybrid_against_exact_f32_and_oracle(head, nin, nout, N):
    """The cached 16-row VJP (its two 64x64 products on split bf16 operands) against the
    exact-f32 uncached VJP on the same head rows (f32 rounding apart) and against the
    float64 J^T g of the oracle at 1e-4."""
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    rng = np.random.default_rng(nin + N)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    kind = {"gauss": _lib.HEAD_GAUSS, "softmax": _lib.HEAD_SOFTMAX, "linear": _lib.HEAD_LINEAR}[head]
    net = MlpNet(nin, nout, kind)
    net.set_flat(th)
    x = _dev(ob)
    # a recording pass writes the activation cache the VJP reads
    if head == "linear":
        tgt = _dev(rng.standard_normal(N))
        gh = torch.zeros(N, dtype=torch.float32, device="cuda")
        part = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        net.rows(_lib.EPI_VFLOSS, x, N, inv_n_global=1.0 / N, target=tgt, ghead=gh, partial=part)
    else:
        oldprob = T.policy_prob(spec, th, ob).astype(np.float32).astype(np.float64)
        act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
        gh = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
        part = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(rng.standard_normal(N)),
                 oldprob=_dev(oldprob), ghead=gh, partial=part)
    outs = {}
    for v, image in (("hyb", None), ("f32", net.image)):
        o = torch.zeros(net.P, dtype=torch.float32, device="cuda")
        net.vjp_flat(x, N, gh, o, image=image)
        outs[v] = o.cpu().numpy().astype(np.float64)
    assert _rel(outs["hyb"], outs["f32"]) < 1e-5
    g = gh.cpu().numpy().astype(np.float64).reshape(N, -1)
    _, acts = T.mlp_forward(spec, th, ob)
    parts = [p.ravel() for p in T.mlp_vjp(spec, th, acts, g[:, :nout])]
    if head == "gauss":
        parts.append(g[:, nout:].sum(axis=0))  # the logstd slot: the rows' own log-std gradients
    want = np.concatenate(parts)
    assert _rel(outs["hyb"], want) < 1e-4
    assert _rel(outs["f32"], want) < 1e-4


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2)])
@pytest.mark.parametrize("N", [1, 33, 3001, 70001])
@pytest.mark.parametrize("cus", [0, 48])
def test_onepass_fisher_product(head, nin, nout, N, cus, monkeypatch):
    """mrl_mlp_fisher_hyb (JVP rows and hybrid VJP side by side in one launch, the head
    rows through LDS) against the two-kernel pair on the same split tangent image (the same
    per-row values, summed over another row partition: f32 rounding apart), against the
    float64 oracle at 1e-4, and bit-identical run to run -- on the whole device and on a
    48-CU subset (the grid and slab rows follow the net's CU count)."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    rng = np.random.default_rng(nin * 13 + N)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    v = rng.standard_normal(spec.P).astype(np.float32)
    net = MlpNet(nin, nout, _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX)
    assert net.fisher_onepass
    net.set_flat(th)
    if cus:
        net.size_for_cus(cus)
    x, vt = _dev(ob), _dev(v)
    a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    gh = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob), ghead=gh,
             partial=partial)
    imgs = net.new_tangent_image()
    net.pack_tangent(vt, imgs)
    assert net.fisher_onepass_applies(x, N, imgs)
    f1 = [torch.full((net.P,), float("nan"), dtype=torch.float32, device="cuda") for _ in range(3)]
    for f in f1:
        assert net.fisher_product(x, N, 1.0 / N, vt, imgs, f)
    torch.cuda.synchronize()
    for f in f1[1:]:
        assert torch.equal(f, f1[0])
    gh2 = torch.full_like(gh, float("nan"))
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh2, tangent=vt, image_t=imgs)
    f2 = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, gh2, f2)
    one, two = f1[0].cpu().numpy().astype(np.float64), f2.cpu().numpy().astype(np.float64)
    assert np.isfinite(one).all()
    assert _rel(one, two) < 1e-5
    want = T.fisher_vector_product(spec, th, v.astype(np.float64), ob)
    assert _rel(one, want) < 1e-4


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2)])  # the static shapes
@pytest.mark.parametrize("N", [1, 33, 3001, 70001])
@pytest.mark.parametrize("cus", [0, 48])
def test_onepass_policy_gradient(head, nin, nout, N, cus, monkeypatch):
    """mrl_mlp_grad_hyb (the SURRGRAD rows of mrl_mlp_rows_split and the hybrid VJP side
    by side in one launch, the head-gradient rows through LDS, trpo.py:42-43) against the
    two-kernel pair: the activation cache it records bit for bit (the same per-row code),
    g to f32 rounding (the same head rows, summed over another row partition), the
    surr / KL / entropy sums to 1e-12; against the float64 oracle at 1e-4; bit-identical
    run to run; the Fisher product that reads its cache equals the one after the pair's."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    rng = np.random.default_rng(nin * 17 + N)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
    if head == "gauss":
        act = act.astype(np.float32).astype(np.float64)
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    v = (0.1 * rng.standard_normal(spec.P)).astype(np.float32)
    monkeypatch.setenv("MRL_GRAD_ONEPASS", "1")
    net = MlpNet(nin, nout, _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX)
    assert net.grad_onepass
    net.set_flat(th)
    if cus:
        net.size_for_cus(cus)
    x, vt, advd, opd = _dev(ob), _dev(v), _dev(adv), _dev(oldprob)
    a = _dev(act, torch.int32 if head == "softmax" else torch.float32)
    ncache = ((N + 31) // 32) * 64 * 64
    imgs = net.new_tangent_image()
    net.pack_tangent(vt, imgs)

    def fisher():
        f = torch.zeros(net.P, device="cuda")
        assert net.fisher_product(x, N, 1.0 / N, vt, imgs, f)
        return f.cpu().numpy().astype(np.float64)

    # the two-kernel pair
    net._cache(N).fill_(float("nan"))
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    gh = torch.full((N * net.gh,), float("nan"), device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=advd, oldprob=opd, ghead=gh, partial=partial)
    s2 = torch.zeros(4, dtype=torch.float64, device="cuda")
    net.reduce_partial(partial, N, s2)
    c2 = net._cache(N)[:ncache].clone()
    g2 = torch.zeros(net.P, device="cuda")
    net.vjp_flat(x, N, gh, g2)
    f2 = fisher()
    # the one launch, three times
    runs = []
    for _ in range(3):
        net._cache(N).fill_(float("nan"))
        g1 = torch.full((net.P,), float("nan"), device="cuda")
        s1 = torch.full((4,), float("nan"), dtype=torch.float64, device="cuda")
        assert net.policy_gradient(x, N, 1.0 / N, a, advd, opd, g1, s1)
        runs.append((g1, s1, net._cache(N)[:ncache].clone()))
    f1 = fisher()
    torch.cuda.synchronize()
    for g1, s1, c1 in runs[1:]:
        assert torch.equal(g1, runs[0][0]) and torch.equal(s1, runs[0][1]) and torch.equal(c1, runs[0][2])
    g1, s1, c1 = (t.cpu().numpy().astype(np.float64) for t in runs[0])
    assert np.array_equal(c1, c2.cpu().numpy().astype(np.float64), equal_nan=True)
    assert np.isfinite(g1).all()
    assert _rel(g1, g2.cpu().numpy().astype(np.float64)) < 1e-5
    np.testing.assert_allclose(s1[:3], s2.cpu().numpy()[:3], rtol=1e-12, atol=1e-12 * np.abs(s1[:3]).max())
    assert s1[3] == 0.0
    np.testing.assert_array_equal(f1, f2)
    want = T.surr_kl_ent(spec, th, ob, act, adv, oldprob)
    np.testing.assert_allclose(np.array([-s1[0] / N, s1[1] / N, s1[2] / N]), want, rtol=1e-4, atol=1e-6)
    assert _rel(g1, T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 1e-4


def _rows_pair(monkeypatch, head, nin, nout, th, build):
    """build(net) on a split-forward net and on an exact-f32 one (MRL_ROWS_SPLIT=0)."""
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    kind = {"gauss": _lib.HEAD_GAUSS, "softmax": _lib.HEAD_SOFTMAX, "linear": _lib.HEAD_LINEAR}[head]
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("MRL_ROWS_SPLIT", flag)
        net = MlpNet(nin, nout, kind)
        assert net.rows_split == (flag == "1")
        net.set_flat(th)
        out.append(build(net))
    return out


@pytest.mark.parametrize("head,nin,nout", CASES)
@pytest.mark.parametrize("N", [1, 33, 3001, 70001])
def test_split_forward_rows(head, nin, nout, N, monkeypatch):
    """mrl_mlp_rows_split (the forward row passes on split bf16 operands) against the
    exact-f32 row kernel (per-row values to f32 rounding: rows 2e-5, loss sums 1e-6, the
    activation cache it writes 2e-6 absolute on tanh outputs) and against the float64
    oracle at 1e-4: prob rows, the TRPO losses, the surrogate-gradient rows and the policy
    gradient from the cache they wrote."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    rng = np.random.default_rng(nin * 3 + N)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
    if head == "gauss":
        act = act.astype(np.float32).astype(np.float64)
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    x, a = _dev(ob), _dev(act, torch.int32 if head == "softmax" else torch.float32)

    def build(net):
        prob = net.forward(x, N).clone()
        partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        gh = torch.full((N * net.gh,), float("nan"), device="cuda")
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
                 ghead=gh, partial=partial)
        sums = torch.zeros(4, dtype=torch.float64, device="cuda")
        net.reduce_partial(partial, N, sums)
        cache = net._cache(N)[: ((N + 31) // 32) * 64 * 64].clone()
        g = torch.zeros(net.P, device="cuda")
        net.vjp_flat(x, N, gh, g)
        lp = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        net.rows(_lib.EPI_LOSSES, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
                 partial=lp)
        ls = torch.zeros(4, dtype=torch.float64, device="cuda")
        net.reduce_partial(lp, N, ls)
        return [t.cpu().numpy().astype(np.float64) for t in (prob, gh, sums, cache, g, ls)]

    (p1, gh1, s1, c1, g1, l1), (p0, gh0, s0, c0, g0, l0) = _rows_pair(monkeypatch, head, nin, nout, th, build)
    np.testing.assert_allclose(p1, p0, rtol=2e-5, atol=2e-6 * np.abs(p0).max())
    np.testing.assert_allclose(gh1, gh0, rtol=2e-5, atol=2e-6 * np.abs(gh0).max())
    # the KL sum is a difference of near-equal terms: f32 rounding of the rows moves it by
    # ~1e-7 of the largest sum, whichever kernel rounds
    np.testing.assert_allclose(s1[:3], s0[:3], rtol=1e-5, atol=1e-6 * np.abs(s0[:3]).max())
    np.testing.assert_allclose(l1[:3], s1[:3], rtol=1e-12, atol=0)  # LOSSES == SURRGRAD's sums
    assert np.abs(c1 - c0).max() < 2e-6
    assert _rel(g1, g0) < 1e-5
    np.testing.assert_allclose(p1, T.policy_prob(spec, th, ob), rtol=2e-5, atol=2e-6)
    want = T.surr_kl_ent(spec, th, ob, act, adv, oldprob)
    np.testing.assert_allclose(np.array([-s1[0] / N, s1[1] / N, s1[2] / N]), want, rtol=1e-4, atol=1e-6)
    assert _rel(g1, T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 1e-4


@pytest.mark.parametrize("nin", [5, 12])
@pytest.mark.parametrize("N", [1, 1500, 70001])
def test_split_forward_value_rows(nin, N, monkeypatch):
    """The value net's passes on split operands: the prediction with the time feature
    (and the feature rows it writes) and the VF loss / gradient rows, against the exact-f32
    kernel and the float64 oracle (core.py:611-617, 648-660)."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    limit = 200.0
    rng = np.random.default_rng(nin + N)
    spec = T.Spec(nin, [64, 64], 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.05 * rng.standard_normal(spec.P)).astype(np.float32).astype(np.float64)
    obs = rng.standard_normal((N, nin - 1)).astype(np.float32)
    ept = rng.integers(0, 200, size=N).astype(np.int32)
    X = np.concatenate([obs.astype(np.float64), (ept / limit).astype(np.float32).astype(np.float64)[:, None]], axis=1)
    y = rng.standard_normal(N).astype(np.float32)
    xo, et, yd = _dev(obs), _dev(ept, torch.int32), _dev(y)

    def build(net):
        feat = torch.full((N, nin), float("nan"), device="cuda")
        v = net.forward(xo, N, ep_t=et, timestep_limit=limit, feat_out=feat).clone()
        xf = feat.clone()
        partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        gh = torch.zeros(N, device="cuda")
        net.rows(_lib.EPI_VFLOSS, xf, N, inv_n_global=1.0 / N, target=yd, ghead=gh, partial=partial)
        sums = torch.zeros(4, dtype=torch.float64, device="cuda")
        net.reduce_partial(partial, N, sums)
        g = torch.zeros(net.P, device="cuda")
        net.vjp_flat(xf, N, gh, g)
        return [t.cpu().numpy().astype(np.float64) for t in (v, xf, gh, sums, g)]

    (v1, f1, gh1, s1, g1), (v0, f0, gh0, s0, g0) = _rows_pair(monkeypatch, "linear", nin, 1, th, build)
    assert np.array_equal(f1, f0)
    np.testing.assert_allclose(f1, X, rtol=0, atol=0)
    np.testing.assert_allclose(v1, v0, rtol=2e-5, atol=2e-6 * np.abs(v0).max())
    np.testing.assert_allclose(gh1, gh0, rtol=2e-5, atol=2e-6 * np.abs(gh0).max())
    np.testing.assert_allclose(s1[0], s0[0], rtol=1e-5)
    assert _rel(g1, g0) < 1e-5
    np.testing.assert_allclose(v1, T.mlp_forward(spec, th, X)[0][:, 0], rtol=2e-5, atol=2e-6)
    loss, gw, mse, l2 = T.vf_loss_grad(spec, th, X, y.astype(np.float64))
    np.testing.assert_allclose(s1[0] / N, mse, rtol=1e-5)
    assert _rel(g1 + 2e-3 * th, gw) < 1e-4


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2), ("gauss", 17, 6)])
def test_cg_update_pack_writes_the_split_tangent_image(head, nin, nout, monkeypatch):
    """mrl_cg_update_pack (the CG update that also writes the next tangent's split image)
    leaves x / r / p / p32 / ax / state bit-identical to mrl_cg_update, and its image is
    mrl_mlp_pack_split's of the new p32 word for word; converged (flag set) it touches
    nothing."""
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, ptr
    from modular_rl_amd.nets import MlpNet
    from modular_rl_amd.trpo import HipTrpoOps
    net = MlpNet(nin, nout, _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX)
    rng = np.random.default_rng(nin)
    P = net.P
    outs = []
    for fused in (False, True):
        ops = HipTrpoOps(net)
        ops.cg_pack = fused
        b = _dev(rng.standard_normal(P) if not outs else outs[0]["b"], torch.float64)
        ops.cg_init(b)
        fv = _dev(np.random.default_rng(5).standard_normal(P))
        ops.tan_image.fill_(float("nan"))
        for _ in range(3):
            ops.cg_update(fv, 1e-3, 1e-10)
        torch.cuda.synchronize()
        outs.append(dict(b=b.cpu().numpy(), **{k: getattr(ops, k).cpu().numpy().copy()
                                             for k in ("x", "r", "p", "p32", "ax", "state", "tan_image")}))
        if fused:
            ref = net.new_tangent_image()
            net.pack_tangent(ops.p32, ref)
            got = ops.tan_image.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, ref.cpu().numpy().view(np.uint32))
            # converged: the update (and its pack) leaves everything as it is
            ops.flag.fill_(1)
            ops.tan_image.fill_(7.0)
            ops.cg_update(fv, 1e-3, 1e-10)
            assert bool((ops.tan_image == 7.0).all())
    for k in ("x", "r", "p", "p32", "ax", "state"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


def test_cg_update_pack_refuses_wide_nets_and_mismatched_sizes(monkeypatch):
    monkeypatch.setenv("MRL_FISHER", "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    net = MlpNet(11, 3, _lib.HEAD_GAUSS)
    lib = _lib.load()
    P = net.P
    z = torch.zeros(P + 8, dtype=torch.float64, device="cuda")
    f = torch.zeros(P + 8, dtype=torch.float32, device="cuda")
    st = torch.zeros(4, dtype=torch.float64, device="cuda")
    fl = torch.zeros(2, dtype=torch.int32, device="cuda")
    img = net.new_tangent_image()
    import ctypes
    args = lambda n: (f.data_ptr(), 1e-3, 1e-10, n, z.data_ptr(), z.data_ptr(), z.data_ptr(), f.data_ptr(),
                      z.data_ptr(), st.data_ptr(), fl.data_ptr(), ctypes.byref(net.desc), img.data_ptr(), None)
    assert lib.mrl_cg_update_pack(*args(P + 1)) == -1  # MRL_E_ARG
    assert lib.mrl_cg_update_pack(*args(9000)) == -2  # MRL_E_UNSUPPORTED
    torch.cuda.synchronize()
