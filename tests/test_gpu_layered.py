"""GPU parity of the layered (tiled MFMA GEMM) MLP path against the float64 oracle:
forward / losses / policy gradient / Fisher product / VF loss-grad for shapes the
fused 64-wide kernels do not cover -- Humanoid 376-512-512-512-17,
odd widths, one hidden layer, n_out > 8 -- plus the [64, 64] shape both paths run."""
import numpy as np
import pytest
import torch

from oracle import trpo_np as T

pytestmark = pytest.mark.gpu

CASES = [
    ("gauss", 11, 3, [64, 64]),
    ("gauss", 376, 17, [512, 512, 512]),
    ("softmax", 6, 5, [100, 50, 30]),
    ("gauss", 20, 9, [130]),
    ("softmax", 40, 12, [256, 96]),
]
IDS = ["hopper64", "humanoid512", "odd", "onelayer", "cat12"]


def _net(head, nin, nout, hid):
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import LayeredMlpNet
    h = {"gauss": _lib.HEAD_GAUSS, "softmax": _lib.HEAD_SOFTMAX, "linear": _lib.HEAD_LINEAR}[head]
    return LayeredMlpNet(nin, nout, h, hid)


def _setup(head, nin, nout, hid, N, seed=0):
    rng = np.random.default_rng(seed)
    spec = T.Spec(nin, hid, nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.02 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    oldth = th + 0.005 * rng.standard_normal(spec.P)
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


def test_make_net_dispatch():
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import LayeredMlpNet, MlpNet, make_net
    assert isinstance(make_net(11, 3, _lib.HEAD_GAUSS, [64, 64]), MlpNet)
    assert isinstance(make_net(376, 17, _lib.HEAD_GAUSS, [512, 512, 512]), LayeredMlpNet)
    assert isinstance(make_net(11, 3, _lib.HEAD_GAUSS, [64, 64], impl="layered"), LayeredMlpNet)
    assert isinstance(make_net(11, 3, _lib.HEAD_GAUSS, [32]), LayeredMlpNet)


@pytest.mark.parametrize("head,nin,nout,hid", CASES, ids=IDS)
@pytest.mark.parametrize("N", [1, 77, 1000])
def test_forward_prob(head, nin, nout, hid, N):
    spec, th, ob, *_ = _setup(head, nin, nout, hid, N)
    net = _net(head, nin, nout, hid)
    net.set_flat(th)
    got = net.forward(_dev(ob), N).cpu().numpy().astype(np.float64)
    want = T.policy_prob(spec, th, ob)
    np.testing.assert_allclose(got, want, rtol=5e-5, atol=5e-6)


@pytest.mark.parametrize("head,nin,nout,hid", CASES, ids=IDS)
def test_losses_and_policy_gradient(head, nin, nout, hid):
    from modular_rl_amd import _lib
    N = 700
    spec, th, ob, act, adv, oldprob = _setup(head, nin, nout, hid, N, seed=1)
    net = _net(head, nin, nout, hid)
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
    # LOSSES-only pass (line search) at another theta leaves the tape alone
    partial.zero_()
    th2 = torch.as_tensor(th * 1.01, dtype=torch.float32).cuda()
    net.rows(_lib.EPI_LOSSES, x, N, inv_n_global=1.0 / N, act=a, adv=_dev(adv), oldprob=_dev(oldprob),
             partial=partial, theta=th2)
    net.reduce_partial(partial, N, sums)
    s = sums.cpu().numpy()
    want2 = T.surr_kl_ent(spec, th2.double().cpu().numpy(), ob, act, adv, oldprob)
    np.testing.assert_allclose(np.array([-s[0] / N, s[1] / N, s[2] / N]), want2, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("head,nin,nout,hid", CASES, ids=IDS)
def test_fisher_vector_product(head, nin, nout, hid):
    from modular_rl_amd import _lib
    N = 600
    spec, th, ob, *_ = _setup(head, nin, nout, hid, N, seed=2)
    rng = np.random.default_rng(5)
    net = _net(head, nin, nout, hid)
    net.set_flat(th)
    x = _dev(ob)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    for rep in range(2):  # the second product reuses the recorded forward tape
        v = rng.standard_normal(spec.P).astype(np.float32)
        vt = _dev(v)
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt)
        net.vjp_flat(x, N, ghead, fv)
        want = T.fisher_vector_product(spec, th, v.astype(np.float64), ob)
        assert _rel(fv.cpu().numpy(), want) < 1e-4, rep


def test_fvp_tape_follows_theta_updates():
    from modular_rl_amd import _lib
    head, nin, nout, hid = "gauss", 11, 3, [96, 48]
    N = 300
    spec, th, ob, *_ = _setup(head, nin, nout, hid, N, seed=4)
    net = _net(head, nin, nout, hid)
    net.set_flat(th)
    x = _dev(ob)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    v = np.random.default_rng(1).standard_normal(spec.P).astype(np.float32)
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=_dev(v))
    th3 = (th * 0.9).astype(np.float32).astype(np.float64)
    net.theta.copy_(_dev(th3))  # in-place update, as TrpoUpdater does
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=_dev(v))
    net.vjp_flat(x, N, ghead, fv)
    want = T.fisher_vector_product(spec, th3, v.astype(np.float64), ob)
    assert _rel(fv.cpu().numpy(), want) < 1e-4


@pytest.mark.parametrize("nin,hid", [(377, [512, 512, 512]), (12, [64, 64]), (30, [200])])
def test_value_forward_and_loss_grad_with_time_feature(nin, hid):
    from modular_rl_amd import _lib
    N, limit = 900, 1000.0
    rng = np.random.default_rng(3)
    spec = T.Spec(nin, hid, 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.02 * rng.standard_normal(spec.P)).astype(np.float32).astype(np.float64)
    obs = rng.standard_normal((N, nin - 1)).astype(np.float32)
    ept = rng.integers(0, 1000, size=N).astype(np.int32)
    X = np.concatenate([obs.astype(np.float64), (ept / limit).astype(np.float32).astype(np.float64)[:, None]], axis=1)
    y = rng.standard_normal(N).astype(np.float32)
    net = _net("linear", nin, 1, hid)
    net.set_flat(th)
    xo, et = _dev(obs), _dev(ept, torch.int32)
    v = net.forward(xo, N, ep_t=et, timestep_limit=limit).cpu().numpy()
    want_v = T.mlp_forward(spec, th, X)[0][:, 0]
    np.testing.assert_allclose(v, want_v, rtol=5e-5, atol=5e-6)
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


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (130, 70, 33), (257, 129, 300), (300, 17, 520), (1024, 512, 512),
                                   (8192, 512, 512), (8192, 512, 376)])
@pytest.mark.parametrize("compute", ["f32", "split"])
def test_gemm_orientations_and_epilogues(M, N, K, compute):
    """mrl_gemm against torch fp64 for every operand orientation and epilogue, on the
    exact-f32 MFMA and on split bf16 operands (MRL_COMPUTE_SPLIT: fp32-accurate); the
    8192-row cases run the 128-column tile the C5 layers use (asserted via
    mrl_gemm_tile_n), the others the narrow 128x32 one."""
    import ctypes
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    _lib.load(require_gpu=True)
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    A2 = torch.randn(M, K, generator=g)
    B2 = torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    H = torch.rand(M, N, generator=g)
    addr = lambda t: ctypes.c_void_p(t.data_ptr())
    cm = _lib.COMPUTE_SPLIT if compute == "split" else _lib.COMPUTE_F32
    bias_d, H_d = bias.cuda(), H.cuda()  # keep the device copies alive while the kernels read them
    for at in (0, 1):
        for bt in (0, 1):
            Ad = (A.t().contiguous() if at else A).cuda()
            Bd = (B.t().contiguous() if bt else B).cuda()
            A2d = (A2.t().contiguous() if at else A2).cuda()
            B2d = (B2.t().contiguous() if bt else B2).cuda()
            lda = M if at else K
            ldb = K if bt else N
            for epi in (_lib.GEMM_STORE, _lib.GEMM_TANH, _lib.GEMM_DTANH):
                C = torch.zeros(M, N, device="cuda")
                d = _lib.GemmDesc(m=M, n=N, k=K, a=addr(Ad), lda=lda, a_trans=at, b=addr(Bd), ldb=ldb, b_trans=bt,
                                  epilogue=epi, a2=addr(A2d), b2=addr(B2d), c=addr(C), ldc=N, bias=addr(bias_d),
                                  h=addr(H_d), ldh=N, compute=cm)
                assert _lib.load().mrl_gemm_tile_n(ctypes.byref(d)) == (128 if M >= 8192 else 32)
                call("mrl_gemm", ctypes.byref(d), None, stream())
                ref = (A.double() @ B.double() + A2.double() @ B2.double() + bias.double())
                scale = ref.abs().max().item()  # fp32 rounding of the pre-activation sets the error scale
                if epi == _lib.GEMM_TANH:
                    ref = torch.tanh(ref)
                elif epi == _lib.GEMM_DTANH:
                    ref = ref * (1 - H.double() ** 2)
                err = (C.cpu().double() - ref).abs().max().item() / max(scale, 1e-30)
                assert err < 1e-5, (at, bt, epi, err)
    # split-K slabs with the ones-row (bias grad) and stride
    Ad = A.t().contiguous().cuda()  # [K, M]: op(A)(i,k) = Ad[k*M + i]  (a_trans = 1)
    Bd = B.cuda()
    S = int(_lib.load().mrl_gemm_slab_splits(K, 4))
    stride = (M + 1) * N + 5
    slab = torch.zeros(S * stride, device="cuda")
    d = _lib.GemmDesc(m=M + 1, n=N, k=K, a=addr(Ad), lda=M, a_trans=1, ones_row=1, b=addr(Bd), ldb=N,
                      epilogue=_lib.GEMM_SLAB, c=addr(slab), ldc=N, splits=4, slab_stride=stride, compute=cm)
    call("mrl_gemm", ctypes.byref(d), None, stream())
    got = slab.view(S, stride)[:, :(M + 1) * N].sum(0).view(M + 1, N).cpu().double()
    ref = torch.cat([A.double(), torch.ones(1, K, dtype=torch.float64)], 0) @ B.double()
    assert (got - ref).abs().max().item() < 1e-4 * max(ref.abs().max().item(), 1.0)


@pytest.mark.parametrize("din", [376, 512])
@pytest.mark.parametrize("compute", ["f32", "split"])
def test_gemm_weight_gradient_slabs_at_production_tile(din, compute):
    """The TN weight-gradient GEMM as the C5 VJP issues it (LayeredMlpNet.vjp_flat):
    dW = X^T G over K = 65,536 rows in 64 split-K slabs, with the bias gradient as the
    ones-row when din is not a multiple of 128 -- >= 160 blocks, so the 128-column tile
    (mrl_gemm_tile_n) -- against the float64 product, summed over the slabs."""
    import ctypes
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    lib = _lib.load(require_gpu=True)
    rows, dout = 65536, 512
    gen = torch.Generator(device="cuda").manual_seed(din)
    X = torch.randn(rows, din, device="cuda", generator=gen)
    G = torch.randn(rows, dout, device="cuda", generator=gen) * 1e-3
    ones = din % 128 != 0
    m = din + ones
    S = int(lib.mrl_gemm_slab_splits(rows, 64))
    stride = m * dout + 7
    slab = torch.full((S * stride,), float("nan"), device="cuda")
    cm = _lib.COMPUTE_SPLIT if compute == "split" else _lib.COMPUTE_F32
    addr = lambda t: ctypes.c_void_p(t.data_ptr())
    d = _lib.GemmDesc(m=m, n=dout, k=rows, a=addr(X), lda=din, a_trans=1, ones_row=int(ones), b=addr(G), ldb=dout,
                      epilogue=_lib.GEMM_SLAB, c=addr(slab), ldc=dout, splits=64, slab_stride=stride, compute=cm)
    assert S == 64 and lib.mrl_gemm_tile_n(ctypes.byref(d)) == 128
    call("mrl_gemm", ctypes.byref(d), None, stream())
    got = slab.view(S, stride)[:, :m * dout].double().sum(0).view(m, dout)
    Xd = X.double()
    if ones:
        Xd = torch.cat([Xd, torch.ones(rows, 1, dtype=torch.float64, device="cuda")], 1)
    ref = Xd.t() @ G.double()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("M,N,ldg,S", [(5000, 17, 34, 3), (1048576, 17, 34, 256), (777, 70, 70, 5), (40, 3, 3, 7)])
def test_colsum_slabs_follow_their_summation_order(M, N, ldg, S):
    """mrl_colsum (the bias / log-std gradient slabs) bit for bit against a float32
    restatement of its order: per slab, wave w (of 4) keeps four accumulators over rows
    r0 + w + 4q + 16j, a tail of rows into the first, then ((s0 + s1) + (s2 + s3)) per wave
    and ((w0 + w1) + (w2 + w3)) per slab -- the batched loads must not change it."""
    import ctypes

    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(M)
    G = rng.standard_normal((M, ldg)).astype(np.float32)
    dG = torch.as_tensor(G).cuda()
    st = (N + 63) // 64 * 64
    slab = torch.full((S * st,), float("nan"), dtype=torch.float32, device="cuda")
    call("mrl_colsum", ctypes.c_void_p(dG.data_ptr()), M, N, ldg, S, ctypes.c_void_p(slab.data_ptr()), st, None,
         stream())
    got = slab.cpu().numpy()
    chunk = (M + S - 1) // S
    for z in range(S):
        r0, r1 = z * chunk, min(M, z * chunk + chunk)
        waves = []
        for w in range(4):
            s = [np.zeros(N, np.float32) for _ in range(4)]
            r = r0 + w
            while r + 12 < r1:
                for q in range(4):
                    s[q] = s[q] + G[r + 4 * q, :N]
                r += 16
            while r < r1:
                s[0] = s[0] + G[r, :N]
                r += 4
            waves.append((s[0] + s[1]) + (s[2] + s[3]))
        want = (waves[0] + waves[1]) + (waves[2] + waves[3])
        np.testing.assert_array_equal(got[z * st:z * st + N], want)


@pytest.mark.parametrize("dtype,ep", [("fp32", True), ("bf16", True), ("bf16", False)])
def test_vf_fit_with_pinned_rows_equals_unpinned(dtype, ep):
    """LbfgsOptimizer.update pins the fit's rows (LayeredMlpNet.pin_input): the tape's
    input ([obs, t/limit] and its bf16 cast) is built once for all evaluations. The
    fitted theta and every stat equal the fit that rebuilds it per evaluation, bit for
    bit; the pin is released after the fit (a later pass over other rows rebuilds)."""
    from modular_rl_amd.nets import LayeredMlpNet
    from modular_rl_amd import _lib
    from modular_rl_amd.vf import LbfgsOptimizer
    from modular_rl_amd.dist import Comm
    N, nin, hid, limit = 3000, 41, [128, 128], 1000.0
    rng = np.random.default_rng(4)
    spec = T.Spec(nin, hid, 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.02 * rng.standard_normal(spec.P)).astype(np.float32)
    obs = _dev(rng.standard_normal((N, nin - 1 if ep else nin)).astype(np.float32))
    ept = _dev(rng.integers(0, 1000, size=N).astype(np.int32), torch.int32) if ep else None
    y = _dev(rng.standard_normal(N).astype(np.float32))
    outs = []
    for pinned in (True, False):
        net = LayeredMlpNet(nin, 1, _lib.HEAD_LINEAR, hid, dtype=dtype)
        net.set_flat(th.astype(np.float64))
        if not pinned:
            net.pin_input = None
        opt = LbfgsOptimizer(net, maxiter=4, comm=Comm())
        info = opt.update((obs, ept, limit, N, y, N))
        assert net._pinned is None and net._pinned_input is None
        outs.append((net.get_flat(), info, opt.n_evals))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1] and outs[0][2] == outs[1][2] > 2
