"""GPU checks of the bf16 throughput mode (MRL_COMPUTE_BF16) through the C ABI.

fp32 is the parity dtype (north_star: 1e-4 relative); bf16 rounds the MFMA operands
(weights, layer inputs, backpropagated rows) to bf16 and accumulates in f32.  Two
bounds per pass:
  * against a float64 numpy emulation of the SAME rounding points (bfr() below):
    only f32 accumulation order, the tanh approximation and the rare bf16 rounding
    flip those cause differ -> rel 3e-3 on sums over rows;
  * against the unrounded float64 oracle: the bf16 bound, rel 3e-2 (8 significant
    bits per operand, errors averaging over K and over rows).
"""
import numpy as np
import pytest
import torch

from oracle import trpo_np as T

pytestmark = pytest.mark.gpu

BF16_EMU_RTOL = 3e-3
BF16_ORACLE_RTOL = 3e-2


def bfr(a):
    """Round to bf16 (RNE) through float32, returned as float64."""
    u = np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


# ---- float64 emulation of csrc/mlp_bf16.hip's rounding points (fused 64-wide net)
def emu_forward(spec, th, x):
    (W0, W1, W2), (b0, b1, b2), _ = spec.split(th)
    xb = bfr(x)
    h1 = bfr(np.tanh(xb @ bfr(W0) + b0))
    h2 = bfr(np.tanh(h1 @ bfr(W1) + b1))
    z = h2 @ W2 + b2  # f32 VALU head on the rounded h2
    return z, (xb, h1, h2)


def emu_vjp(spec, th, acts, G, gls=None):
    (W0, W1, W2), _, _ = spec.split(th)
    xb, h1, h2 = acts
    Gb = bfr(G)
    ga2 = bfr((Gb @ bfr(W2).T) * (1 - h2 ** 2))
    ga1 = (ga2 @ bfr(W1).T) * (1 - h1 ** 2)
    out = [xb.T @ bfr(ga1), ga1.sum(0), h1.T @ ga2, ga2.sum(0), h2.T @ Gb, G.sum(0)]
    if gls is not None:
        out.append(gls)
    return T.flatten(out)


def emu_jvp(spec, th, v, acts):
    (W0, W1, W2), _, _ = spec.split(th)
    (dW0, dW1, dW2), (db0, db1, db2), _ = spec.split(v)
    xb, h1, h2 = acts
    dh1 = bfr((xb @ bfr(dW0) + db0) * (1 - h1 ** 2))
    da2 = (dh1 @ bfr(W1) + h1 @ bfr(dW1) + db1) * (1 - h2 ** 2)
    return da2 @ W2 + h2 @ dW2 + db2


def _setup(head, nin, nout, N, seed):
    rng = np.random.default_rng(seed)
    spec = T.Spec(nin, [64, 64], nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    return rng, spec, th, ob


def _net(head, nin, nout, impl="fused"):
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import make_net
    h = {"gauss": _lib.HEAD_GAUSS, "softmax": _lib.HEAD_SOFTMAX, "linear": _lib.HEAD_LINEAR}[head]
    return make_net(nin, nout, h, [64, 64], impl=impl, dtype="bf16")


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


CASES = [("gauss", 11, 3), ("softmax", 4, 2), ("gauss", 17, 6), ("softmax", 20, 5)]


@pytest.mark.parametrize("head,nin,nout", CASES)
def test_bf16_forward_prob(head, nin, nout):
    N = 3001
    _, spec, th, ob = _setup(head, nin, nout, N, 0)
    net = _net(head, nin, nout)
    net.set_flat(th)
    got = net.forward(_dev(ob), N).cpu().numpy().astype(np.float64)
    z, _ = emu_forward(spec, th, ob)
    emu = T.head_prob(spec, th, z)
    want = T.policy_prob(spec, th, ob)
    np.testing.assert_allclose(got, emu, rtol=BF16_EMU_RTOL, atol=1e-3)
    assert _rel(got, want) < BF16_ORACLE_RTOL


@pytest.mark.parametrize("head,nin,nout", CASES)
def test_bf16_fisher_vector_product(head, nin, nout):
    from modular_rl_amd import _lib
    N = 4000
    rng, spec, th, ob = _setup(head, nin, nout, N, 2)
    v = rng.standard_normal(spec.P).astype(np.float32).astype(np.float64)
    net = _net(head, nin, nout)
    net.set_flat(th)
    x, vt = _dev(ob), _dev(v)
    imgt = torch.zeros_like(net.image)
    net.pack(theta=vt, image=imgt, fwd_only=True)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    got = {}
    for cached in (False, True):
        if cached:  # a recording pass at theta writes the bf16 activation cache
            part = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
            adv = _dev(rng.standard_normal(N))
            prob = _dev(T.policy_prob(spec, th, ob))
            act = _dev(rng.integers(0, nout, N), torch.int32) if head == "softmax" else _dev(ob[:, :nout] * 0.1)
            gtmp = torch.zeros_like(ghead)
            net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gtmp,
                     partial=part)
        else:
            net.use_cache = False
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt, image_t=imgt)
        fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
        net.vjp_flat(x, N, ghead, fv)
        got[cached] = fv.cpu().numpy().astype(np.float64)
        net.use_cache = True
    # emulation: the metric rows from the emulated JVP, then the emulated VJP
    z, acts = emu_forward(spec, th, ob)
    dz = emu_jvp(spec, th, v, acts)
    if head == "softmax":
        p = T.softmax(z)
        G = p * (dz - (p * dz).sum(1, keepdims=True)) / N
        emu = emu_vjp(spec, th, acts, G)
    else:
        _, _, ls = spec.split(th)
        _, _, dls = spec.split(v)
        emu = emu_vjp(spec, th, acts, dz / np.exp(2 * ls)[None, :] / N, 2.0 * dls)
    want = T.fisher_vector_product(spec, th, v, ob)
    for cached, fv in got.items():
        assert _rel(fv, emu) < BF16_EMU_RTOL, (cached, _rel(fv, emu))
        assert _rel(fv, want) < BF16_ORACLE_RTOL, (cached, _rel(fv, want))
    # the cached pass reads exactly the activations the uncached one recomputes
    assert _rel(got[True], got[False]) < 1e-6


@pytest.mark.parametrize("head,nin,nout", CASES[:2])
def test_bf16_losses_and_policy_gradient(head, nin, nout):
    from modular_rl_amd import _lib
    N = 5000
    rng, spec, th, ob = _setup(head, nin, nout, N, 1)
    oldth = th + 0.01 * rng.standard_normal(spec.P)
    oldprob = T.policy_prob(spec, oldth, ob).astype(np.float32).astype(np.float64)
    noise = rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N)
    act = T.sample(spec, oldprob, noise)
    if head == "gauss":
        act = act.astype(np.float32).astype(np.float64)
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
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
    np.testing.assert_allclose(losses, want, rtol=BF16_ORACLE_RTOL, atol=2e-3)
    # gradient: the emulated VJP of the kernel's own head rows, and the oracle
    z, acts = emu_forward(spec, th, ob)
    gh = ghead.cpu().numpy().astype(np.float64).reshape(N, -1)
    if head == "softmax":
        emu = emu_vjp(spec, th, acts, gh)
    else:
        emu = emu_vjp(spec, th, acts, gh[:, :nout], gh[:, nout:].sum(0))
    assert _rel(g.cpu().numpy(), emu) < BF16_EMU_RTOL
    assert _rel(g.cpu().numpy(), T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 5e-2


def test_bf16_value_loss_grad_with_time_feature():
    from modular_rl_amd import _lib
    N, nin, limit = 3000, 12, 200.0
    rng = np.random.default_rng(3)
    spec = T.Spec(nin, [64, 64], 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.05 * rng.standard_normal(spec.P)).astype(np.float32)
    th = th.astype(np.float64)
    ob = rng.standard_normal((N, nin - 1)).astype(np.float32).astype(np.float64)
    ept = rng.integers(0, 200, N)
    X = np.concatenate([ob, (ept / limit)[:, None]], axis=1)
    y = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    net = _net("linear", nin, 1)
    net.set_flat(th)
    x, et = _dev(ob), _dev(ept, torch.int32)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    ghead = torch.zeros(N, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_VFLOSS, x, N, ep_t=et, timestep_limit=limit, inv_n_global=1.0 / N, target=_dev(y),
             ghead=ghead, partial=partial)
    g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, g, ep_t=et, timestep_limit=limit)
    z, acts = emu_forward(spec, th, X)
    emu = emu_vjp(spec, th, acts, 2.0 * (z - y[:, None]) / N)
    _, want_g, _, _ = T.vf_loss_grad(spec, th, X, y)
    want_g = want_g - 2.0 * T.VF_L2 * th  # the kernel's part: the MSE gradient (L2 is added on the host)
    assert _rel(g.cpu().numpy(), emu) < BF16_EMU_RTOL
    assert _rel(g.cpu().numpy(), want_g) < BF16_ORACLE_RTOL


def test_bf16_gemm_exact_on_rounded_operands():
    """mrl_gemm with MRL_COMPUTE_BF16 == the float64 product of the bf16-rounded
    operands up to f32 accumulation (all four orientations, K tail, both tile widths)."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(7)
    for (M, N, K) in [(300, 200, 77), (1000, 24, 512), (64, 512, 130)]:
        for at in (0, 1):
            for bt in (0, 1):
                A = rng.standard_normal((K, M) if at else (M, K)).astype(np.float32)
                B = rng.standard_normal((N, K) if bt else (K, N)).astype(np.float32)
                C = torch.zeros(M * N, dtype=torch.float32, device="cuda")
                dA, dB = _dev(A), _dev(B)
                g = _lib.GemmDesc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=A.shape[1], a_trans=at,
                                  b=ctypes.c_void_p(dB.data_ptr()), ldb=B.shape[1], b_trans=bt,
                                  epilogue=_lib.GEMM_STORE, c=ctypes.c_void_p(C.data_ptr()), ldc=N,
                                  compute=_lib.COMPUTE_BF16)
                call("mrl_gemm", ctypes.byref(g), None, stream())
                opA = bfr(A.T if at else A)
                opB = bfr(B.T if bt else B)
                want = opA @ opB
                got = C.cpu().numpy().reshape(M, N).astype(np.float64)
                err = np.abs(got - want).max() / np.abs(want).max()
                assert err < 1e-5, (M, N, K, at, bt, err)


def _bf16_dev(a, ld):
    """float array [r, c] -> device bf16 bits [r, ld] (RNE, zero padding) via mrl_cast_rows_bf16."""
    import ctypes

    from modular_rl_amd._lib import call, stream
    x = _dev(np.ascontiguousarray(a, dtype=np.float32))
    y = torch.zeros(a.shape[0] * ld, dtype=torch.int16, device="cuda")
    call("mrl_cast_rows_bf16", ctypes.c_void_p(x.data_ptr()), a.shape[0], a.shape[1], a.shape[1],
         ctypes.c_void_p(y.data_ptr()), ld, stream())
    return y


def _bf16_host(y, rows, ld, cols):
    b = y.cpu().numpy().view(np.uint16).astype(np.uint32).reshape(rows, ld)[:, :cols] << 16
    return b.view(np.float32).astype(np.float64)


@pytest.mark.parametrize("epi", ["store", "tanh", "dtanh"])
def test_bf16_operand_gemm_nn_bt(epi):
    """mrl_gemm_bf16 (bf16 operands in memory, B as its transpose image from
    mrl_pack_w_bf16) == the float64 product of the same bf16 operands up to f32
    accumulation; single and dual products, K tails, both tile widths, f32 and bf16
    outputs."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(3)
    E = {"store": _lib.GEMM_STORE, "tanh": _lib.GEMM_TANH, "dtanh": _lib.GEMM_DTANH}[epi]
    for (M, N, K, dual) in [(300, 200, 77, False), (1000, 17, 512, True), (129, 512, 130, True)]:
        ldk = (K + 7) // 8 * 8
        A, A2 = rng.standard_normal((M, K)), rng.standard_normal((M, K))
        W, W2 = rng.standard_normal((K, N)) * 0.1, rng.standard_normal((K, N)) * 0.1
        bias = rng.standard_normal(N).astype(np.float32)
        H = np.tanh(rng.standard_normal((M, N)))
        dA, dA2, dH = _bf16_dev(A, ldk), _bf16_dev(A2, ldk), _bf16_dev(H, N)
        dW, dW2 = _dev(W.astype(np.float32)), _dev(W2.astype(np.float32))
        Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        Bt2 = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        call("mrl_pack_w_bf16", ctypes.c_void_p(dW.data_ptr()), K, N, 1, ctypes.c_void_p(Bt.data_ptr()), ldk, stream())
        call("mrl_pack_w_bf16", ctypes.c_void_p(dW2.data_ptr()), K, N, 1, ctypes.c_void_p(Bt2.data_ptr()), ldk,
             stream())
        db = _dev(bias)
        want = bfr(A) @ bfr(W)
        if dual:
            want = want + bfr(A2) @ bfr(W2)
        want = want + bias.astype(np.float64)
        if epi == "tanh":
            want = np.tanh(want)
        elif epi == "dtanh":
            hb = bfr(H)
            want = want * (1.0 - hb * hb)
        for out_bf in (0, 1):
            C = torch.zeros(M * N, dtype=torch.int16 if out_bf else torch.float32, device="cuda")
            g = _lib.GemmBf16Desc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=ldk,
                                  bt=ctypes.c_void_p(Bt.data_ptr()), ldb=ldk,
                                  a2=ctypes.c_void_p(dA2.data_ptr()) if dual else None,
                                  bt2=ctypes.c_void_p(Bt2.data_ptr()) if dual else None,
                                  c=ctypes.c_void_p(C.data_ptr()), ldc=N, c_bf16=out_bf, epilogue=E,
                                  bias=ctypes.c_void_p(db.data_ptr()), h=ctypes.c_void_p(dH.data_ptr()), ldh=N)
            call("mrl_gemm_bf16", ctypes.byref(g), None, stream())
            got = _bf16_host(C, M, N, N) if out_bf else C.cpu().numpy().reshape(M, N).astype(np.float64)
            err = np.abs(got - want).max() / np.abs(want).max()
            assert err < (8e-3 if out_bf else 2e-5), (M, N, K, dual, out_bf, err)


def test_bf16_operand_gemm_tn_slabs():
    """mrl_gemm_bf16_tn: split-K weight-gradient slabs of two bf16 row-major operands,
    with and without the ones-column (bias gradient), summed over the slabs, equal the
    float64 product of the bf16 operands."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(5)
    for (R, din, dout, ones) in [(3000, 376, 512, True), (2500, 512, 17, False), (777, 96, 80, True)]:
        lda, ldb = (din + 7) // 8 * 8, (dout + 7) // 8 * 8
        X, G = rng.standard_normal((R, din)), rng.standard_normal((R, dout))
        dX, dG = _bf16_dev(X, lda), _bf16_dev(G, ldb)
        M = din + (1 if ones else 0)
        S = int(_lib.load().mrl_gemm_slab_splits(R, 64))
        slab = torch.full((S * M * dout,), float("nan"), dtype=torch.float32, device="cuda")
        g = _lib.GemmBf16TnDesc(m=M, n=dout, k=R, a=ctypes.c_void_p(dX.data_ptr()), lda=lda,
                                b=ctypes.c_void_p(dG.data_ptr()), ldb=ldb, ones_row=int(ones), splits=64,
                                slab=ctypes.c_void_p(slab.data_ptr()), slab_stride=M * dout, ldc=dout)
        call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())
        got = slab.cpu().numpy().reshape(S, M, dout).astype(np.float64).sum(0)
        Xb = bfr(X)
        if ones:
            Xb = np.concatenate([Xb, np.ones((R, 1))], axis=1)
        want = Xb.T @ bfr(G)
        err = np.abs(got - want).max() / np.abs(want).max()
        assert err < 2e-5, (R, din, dout, ones, err)


def test_bf16_tn_big_tiles_equal_tiled(monkeypatch):
    """The 256 x 256 LDS-DMA TN kernel (split-K slabs, transposing reads of swizzled
    images) writes the same weight-gradient slab rows as the 128 x 128 kernel bit for bit
    (same per-slab k order); its ones-row (bias gradient: one selector MFMA per k-step in
    row tile 0's blocks, another summation order) and every row hold the float64 sums.  Ragged rows (slab and stage tails), m / n tails (376 = one full and one
    partial tile, 300), with and without the ones-row, slab counts 64 and 7."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(8)
    for (R, din, dout, ones, splits) in [(40000, 512, 512, True, 64), (33333, 376, 512, True, 64),
                                         (5000, 512, 300, False, 7), (1000, 256, 256, True, 64)]:
        lda, ldb = (din + 7) // 8 * 8, (dout + 7) // 8 * 8
        X, G = rng.standard_normal((R, din)), rng.standard_normal((R, dout))
        dX, dG = _bf16_dev(X, lda), _bf16_dev(G, ldb)
        M = din + (1 if ones else 0)
        S = int(_lib.load().mrl_gemm_slab_splits(R, splits))
        outs = []
        for big in ("0", "1"):
            monkeypatch.setenv("MRL_GEMM_TN_BIG", big)
            slab = torch.full((S * M * dout,), float("nan"), dtype=torch.float32, device="cuda")
            g = _lib.GemmBf16TnDesc(m=M, n=dout, k=R, a=ctypes.c_void_p(dX.data_ptr()), lda=lda,
                                    b=ctypes.c_void_p(dG.data_ptr()), ldb=ldb, ones_row=int(ones), splits=splits,
                                    slab=ctypes.c_void_p(slab.data_ptr()), slab_stride=M * dout, ldc=dout)
            call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())
            torch.cuda.synchronize()
            outs.append(slab.view(S, M, dout))
        assert torch.equal(outs[0][:, :din], outs[1][:, :din]), (R, din, dout)
        got = outs[1].cpu().numpy().astype(np.float64).sum(0)
        Xb = bfr(X)
        if ones:
            Xb = np.concatenate([Xb, np.ones((R, 1))], axis=1)
        want = Xb.T @ bfr(G)
        err = np.abs(got - want).max() / np.abs(want).max()
        assert err < 2e-5, (R, din, dout, ones, err)


@pytest.mark.parametrize("head,nin,nout", [("gauss", 40, 9), ("softmax", 30, 4)])
def test_bf16_layered_fvp_and_gradient(head, nin, nout):
    """Layered GEMM path (hid 96,80) in bf16: Fisher product and gradient at the bf16 bound."""
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import make_net
    N = 3000
    rng = np.random.default_rng(11)
    hid = [96, 80]
    spec = T.Spec(nin, hid, nout, head)
    th = (T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)).astype(np.float32)
    th = th.astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    h = _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX
    net = make_net(nin, nout, h, hid, impl="layered", dtype="bf16")
    net.set_flat(th)
    v = rng.standard_normal(spec.P).astype(np.float32).astype(np.float64)
    x, vt = _dev(ob), _dev(v)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt)
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, fv)
    want = T.fisher_vector_product(spec, th, v, ob)
    assert _rel(fv.cpu().numpy(), want) < BF16_ORACLE_RTOL


def test_bf16_layered_humanoid_shape():
    """C5's net (376-512-512-512-17, DiagGauss) on the bf16 tape: the K = 376 first
    layer (input rows cast with zero padding), the 512-wide layers whose bias gradient
    needs an extra ones-row tile (din % 128 == 0), the 17-wide head; Fisher product,
    policy gradient and the forward against the float64 oracle at the bf16 bound."""
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import make_net
    N, nin, nout, hid = 1500, 376, 17, [512, 512, 512]
    rng = np.random.default_rng(13)
    spec = T.Spec(nin, hid, nout, "gauss")
    th = (T.mlp_init(rng, spec.shapes, True) + 0.02 * rng.standard_normal(spec.P)).astype(np.float32)
    th = th.astype(np.float64)
    ob = rng.standard_normal((N, nin)).astype(np.float32).astype(np.float64)
    net = make_net(nin, nout, _lib.HEAD_GAUSS, hid, impl="layered", dtype="bf16")
    assert net.tape_bf16
    net.set_flat(th)
    x = _dev(ob)
    # forward (prob rows: mean, std)
    out = net.forward(x, N).cpu().numpy().astype(np.float64)
    z, _ = T.mlp_forward(spec, th, ob)
    assert _rel(out[:, :nout], z) < BF16_ORACLE_RTOL
    # Fisher product
    v = rng.standard_normal(spec.P).astype(np.float32).astype(np.float64)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=_dev(v))
    fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, fv)
    assert _rel(fv.cpu().numpy(), T.fisher_vector_product(spec, th, v, ob)) < BF16_ORACLE_RTOL
    # policy gradient of the surrogate (as test_bf16_losses_and_policy_gradient)
    oldth = th + 0.01 * rng.standard_normal(spec.P)
    oldprob = T.policy_prob(spec, oldth, ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout))).astype(np.float32).astype(np.float64)
    adv = rng.standard_normal(N).astype(np.float32).astype(np.float64)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=_dev(act), adv=_dev(adv), oldprob=_dev(oldprob),
             ghead=ghead, partial=partial)
    g = torch.zeros(net.P, dtype=torch.float32, device="cuda")
    net.vjp_flat(x, N, ghead, g)
    assert _rel(g.cpu().numpy(), T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 5e-2


def test_bf16_fisher_product_full_c2_size():
    """C2 at its full size (CartPole net 4-64-64-2, bf16, 4096 x 1024 = 4,194,304 rows):
    the cached Fisher product against the float64 oracle at the bf16 bound, cached ==
    uncached, F(2v) == 2 F(v) bit for bit (scaling by 2 is exact through every rounding
    point) and the symmetry w^T F v = v^T F w (size-independent properties)."""
    from modular_rl_amd import _lib
    N = 4096 * 1024
    head, nin, nout = "softmax", 4, 2
    rng, spec, th, ob = _setup(head, nin, nout, N, 9)
    net = _net(head, nin, nout)
    net.set_flat(th)
    x = _dev(ob)
    ghead = torch.zeros(N * net.gh, dtype=torch.float32, device="cuda")

    def fvp(v, cached=True):
        vt = _dev(v)
        imgt = torch.zeros_like(net.image)
        net.pack(theta=vt, image=imgt, fwd_only=True)
        net.use_cache = cached
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=vt, image_t=imgt)
        fv = torch.zeros(net.P, dtype=torch.float32, device="cuda")
        net.vjp_flat(x, N, ghead, fv)
        net.use_cache = True
        return fv.cpu().numpy().astype(np.float64)

    part = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=_dev(rng.integers(0, nout, N), torch.int32),
             adv=_dev(rng.standard_normal(N)), oldprob=_dev(T.policy_prob(spec, th, ob)), ghead=torch.zeros_like(ghead),
             partial=part)  # the recording pass: writes the bf16 activation cache
    v = rng.standard_normal(spec.P).astype(np.float32).astype(np.float64)
    w = rng.standard_normal(spec.P).astype(np.float32).astype(np.float64)
    fv, fw = fvp(v), fvp(w)
    assert np.array_equal(fvp(2.0 * v), 2.0 * fv)
    assert _rel(fvp(v, cached=False), fv) < 1e-6
    a, b = w @ fv, v @ fw
    assert abs(a - b) <= 1e-3 * max(abs(a), abs(b)), (a, b)
    want = T.fisher_vector_product(spec, th, v, ob)
    assert _rel(fv, want) < BF16_ORACLE_RTOL, _rel(fv, want)


@pytest.mark.parametrize("env_id", ["CartPole-v0", "Hopper-v2"])
def test_bf16_persistent_rollout_full_width_equals_step_launches(env_id):
    """bf16 mode at the C2 / C3 env count (4096 envs = 64 blocks: the full cross-block
    hand-off of the persistent launch with the bf16 forward): the persistent launch and
    T step launches give bit-identical trajectories, filter and env state."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.envs import make
    env = make(env_id)
    cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=4096, horizon=24, seed=6, mlp_dtype="bf16")
    outs = []
    for persistent in (False, True):
        # one agent each (the running filter belongs to the agent), same seed and policy
        agent = TrpoAgent(env.observation_space, env.action_space, cfg)
        col = agent.make_collector(env, cfg)
        col.persistent = persistent
        got = []
        for _ in range(2):
            b = col.collect()
            if persistent:
                col.check()
            got += [t.clone() for t in (b.obs, b.act, b.prob, b.rew, b.flags, b.ep_t)]
        got += [col.filter_state[:col.FS].clone(), col.env_state.clone(), col.env_int.clone(),
                agent.policy.net.theta.clone()]
        outs.append(got)
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("env_id", ["CartPole-v0", "Hopper-v2"])
def test_bf16_rollout_prob_rows_equal_update_forward(env_id):
    """bf16 mode: the rollout's fused forward rounds W0, W1, x, h1, h2 like
    mrl_mlp_rows_bf16, so the prob rows it stores (the update's oldprob) equal the
    update's own bf16 forward on the stored observations up to f32 summation order."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.envs import make
    env = make(env_id)
    cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=256, horizon=32, seed=5, mlp_dtype="bf16")
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    net = agent.policy.net
    assert net.dtype == "bf16"
    col = agent.make_collector(env, cfg)
    b = col.collect()
    got = b.prob.reshape(b.n, -1)
    fwd = net.forward(b.obs, b.n).reshape(b.n, -1)
    err = (got - fwd).abs().max().item() / fwd.abs().max().item()
    assert err < 2e-5, err
    # and the fp32 policy's rows differ from them at bf16 scale (the rounding is real)
    net32 = agent.baseline.net.__class__(net.n_in, net.n_out, net.head)
    net32.set_flat(net.get_flat())
    d32 = (net32.forward(b.obs, b.n).reshape(b.n, -1) - fwd).abs().max().item() / fwd.abs().max().item()
    assert d32 > 1e-4, d32


@pytest.mark.parametrize("hid", [[128, 64], [256, 512]])  # 512: the head's contiguous-run loads
def test_bf16_humanoid_rollout_hidden_rows_on_bf16_gemms(hid):
    """bf16 mode, Humanoid (wave-per-env step, head fused into the step): the rollout's
    hidden layers run on mrl_gemm_bf16 with bf16 rows (mrl_rollout_act_head_bf16), the
    same kernels and rounding points as the update's bf16 tape, so the prob rows the
    rollout stores equal the update's forward on the stored observations up to the
    head's f32 summation order."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=256, horizon=16, seed=3, mlp_dtype="bf16",
               hid_sizes=hid)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    net = agent.policy.net
    col = agent.make_collector(env, cfg)
    assert col.hidden_b16
    b = col.collect()
    got = b.prob.reshape(b.n, -1)
    fwd = net.forward(b.obs, b.n).reshape(b.n, -1)
    err = (got - fwd).abs().max().item() / fwd.abs().max().item()
    assert err < 2e-5, err
    assert torch.isfinite(got).all()


def test_bf16_trpo_learns_cartpole():
    """C2's throughput mode end to end: TRPO with every MLP pass in bf16 still learns."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.core import run_policy_gradient_algorithm
    from modular_rl_amd.envs import make
    env = make("CartPole-v0")
    cfg = dict(timestep_limit=env.spec.max_episode_steps, gamma=0.99, lam=0.97, max_kl=0.01, cg_damping=0.1,
               n_envs=128, horizon=200, seed=1, n_iter=12, mlp_dtype="bf16")
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    assert agent.policy.net.dtype == "bf16" and agent.baseline.net.dtype == "bf16"
    seen = []
    run_policy_gradient_algorithm(env, agent, usercfg=cfg, callback=seen.append)
    assert len(seen) == 12
    assert all(s["pol_kl_after"] <= 2.0 * 0.01 for s in seen)
    assert seen[-1]["EpRewMean"] > 1.5 * seen[0]["EpRewMean"], (seen[0]["EpRewMean"], seen[-1]["EpRewMean"])


@pytest.mark.parametrize("epi", ["store", "tanh", "dtanh"])
def test_bf16_streaming_gemm_equals_tiled(epi, monkeypatch):
    """The streaming NN kernel (tall M, K 257..512: Bt slice resident in LDS, A streamed
    one chunk ahead) against the tiled kernel on the same operands, bit for bit, and
    against the float64 product: row tails (M not a multiple of 256), K tails inside
    lda (377 -> 384, zero padding) and at lda (376: the last k-step half past lda is
    masked, not read), N tails (200: a partial column slice), single / dual, f32 / bf16
    outputs."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(11)
    E = {"store": _lib.GEMM_STORE, "tanh": _lib.GEMM_TANH, "dtanh": _lib.GEMM_DTANH}[epi]
    for (M, N, K, ldk, dual) in [(70001, 512, 512, 512, False), (40000, 512, 512, 512, True),
                                 (33333, 200, 376, 376, False), (35000, 512, 377, 384, True)]:
        A, A2 = rng.standard_normal((M, K)), rng.standard_normal((M, K))
        W, W2 = rng.standard_normal((K, N)) * 0.05, rng.standard_normal((K, N)) * 0.05
        bias = rng.standard_normal(N).astype(np.float32)
        H = np.tanh(rng.standard_normal((M, N)))
        dA, dA2, dH = _bf16_dev(A, ldk), _bf16_dev(A2, ldk), _bf16_dev(H, N)
        Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        Bt2 = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        for w, bt in ((W, Bt), (W2, Bt2)):
            dw = _dev(w.astype(np.float32))
            call("mrl_pack_w_bf16", ctypes.c_void_p(dw.data_ptr()), K, N, 1, ctypes.c_void_p(bt.data_ptr()), ldk,
                 stream())
        db = _dev(bias)
        for out_bf in (0, 1):
            outs = []
            for min_m in ("0", "1"):  # 0: the tiled kernel; 1: streaming for every M
                monkeypatch.setenv("MRL_GEMM_BIG_MIN_M", "0")
                monkeypatch.setenv("MRL_GEMM_STREAM_MIN_M", min_m)
                C = torch.full((M * N,), -7, dtype=torch.int16, device="cuda") if out_bf else \
                    torch.full((M * N,), float("nan"), dtype=torch.float32, device="cuda")
                g = _lib.GemmBf16Desc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=ldk,
                                      bt=ctypes.c_void_p(Bt.data_ptr()), ldb=ldk,
                                      a2=ctypes.c_void_p(dA2.data_ptr()) if dual else None,
                                      bt2=ctypes.c_void_p(Bt2.data_ptr()) if dual else None,
                                      c=ctypes.c_void_p(C.data_ptr()), ldc=N, c_bf16=out_bf, epilogue=E,
                                      bias=ctypes.c_void_p(db.data_ptr()), h=ctypes.c_void_p(dH.data_ptr()), ldh=N)
                call("mrl_gemm_bf16", ctypes.byref(g), None, stream())
                torch.cuda.synchronize()
                outs.append(C)
            assert torch.equal(outs[0], outs[1]), (M, N, K, dual, out_bf)
            if not out_bf:
                f32_out = outs[1]
        rows = rng.choice(M, 300, replace=False)
        rows[0] = M - 1
        want = bfr(A[rows]) @ bfr(W)
        if dual:
            want = want + bfr(A2[rows]) @ bfr(W2)
        want = want + bias.astype(np.float64)
        if epi == "tanh":
            want = np.tanh(want)
        elif epi == "dtanh":
            hb = bfr(H[rows])
            want = want * (1.0 - hb * hb)
        got = f32_out.cpu().numpy().reshape(M, N)[rows].astype(np.float64)
        assert np.abs(got - want).max() / np.abs(want).max() < 2e-5, (M, N, K, dual)


@pytest.mark.parametrize("epi", ["store", "tanh"])
def test_bf16_small_m_gemm_equals_tiled(epi, monkeypatch):
    """The whole-K 64 x 64 kernel for small M (the Humanoid rollout's per-step layers:
    K quarters staged by LDS-DMA, fragment reads as inline asm) against the tiled kernel,
    bit for bit, and the float64 product: M 1024 and ragged (1000, 37), K 512 / 376 (the
    376-d obs) / 200 (a partial last quarter) / 17 (one chunk past K), N 512 / 200 / 64,
    f32 / bf16 outputs, with bias."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(21)
    E = {"store": _lib.GEMM_STORE, "tanh": _lib.GEMM_TANH}[epi]
    monkeypatch.setenv("MRL_GEMM_STREAM_MIN_M", "0")
    monkeypatch.setenv("MRL_GEMM_BIG_MIN_M", "0")
    for (M, N, K) in [(1024, 512, 512), (1024, 512, 376), (1000, 200, 200), (37, 64, 17), (4096, 512, 512)]:
        ldk = (K + 7) // 8 * 8
        A = rng.standard_normal((M, K))
        W = rng.standard_normal((K, N)) * 0.05
        bias = rng.standard_normal(N).astype(np.float32)
        dA = _bf16_dev(A, ldk)
        Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        dw = _dev(W.astype(np.float32))
        call("mrl_pack_w_bf16", ctypes.c_void_p(dw.data_ptr()), K, N, 1, ctypes.c_void_p(Bt.data_ptr()), ldk, stream())
        db = _dev(bias)
        for out_bf in (0, 1):
            outs = []
            for small in ("0", "8192"):
                monkeypatch.setenv("MRL_GEMM_SMALL_MAX_M", small)
                C = torch.full((M * N,), -7, dtype=torch.int16, device="cuda") if out_bf else \
                    torch.full((M * N,), float("nan"), dtype=torch.float32, device="cuda")
                g = _lib.GemmBf16Desc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=ldk,
                                      bt=ctypes.c_void_p(Bt.data_ptr()), ldb=ldk, c=ctypes.c_void_p(C.data_ptr()),
                                      ldc=N, c_bf16=out_bf, epilogue=E, bias=ctypes.c_void_p(db.data_ptr()))
                call("mrl_gemm_bf16", ctypes.byref(g), None, stream())
                torch.cuda.synchronize()
                outs.append(C)
            diff = (outs[0] != outs[1]).sum().item()
            assert diff == 0, (M, N, K, out_bf, diff)
            if not out_bf:
                ab = np.asarray(torch.tensor(A, dtype=torch.float32).to(torch.bfloat16).to(torch.float64))
                wb = np.asarray(torch.tensor(W, dtype=torch.float32).to(torch.bfloat16).to(torch.float64))
                want = ab @ wb + bias
                if epi == "tanh":
                    want = np.tanh(want)
                got = outs[1].cpu().numpy().reshape(M, N).astype(np.float64)
                assert np.abs(got - want).max() / np.abs(want).max() < 2e-5, (M, N, K)


@pytest.mark.parametrize("epi", ["store", "tanh", "dtanh"])
def test_bf16_big_tile_gemm_equals_tiled(epi, monkeypatch):
    """The 256 x 256 LDS-DMA NN kernel (persistent, four 32-deep K stages, XOR-swizzled
    stage images) against the 128 x 128 tiled kernel, bit for bit, and against the
    float64 product: row tails (M not a multiple of 256, fewer row tiles than a round),
    K tails at lda (376: the chunks past K read the zero block) and inside lda (377 ->
    384), N tails (200, 300: partial column tiles, clamped Bt rows), single / dual,
    f32 / bf16 outputs, and two launches of the same call (deterministic)."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(12)
    E = {"store": _lib.GEMM_STORE, "tanh": _lib.GEMM_TANH, "dtanh": _lib.GEMM_DTANH}[epi]
    monkeypatch.setenv("MRL_GEMM_STREAM_MIN_M", "0")
    for (M, N, K, ldk, dual) in [(70001, 512, 512, 512, False), (40000, 512, 512, 512, True),
                                 (3333, 200, 376, 376, False), (35000, 300, 377, 384, True),
                                 (100000, 512, 376, 376, True)]:
        A, A2 = rng.standard_normal((M, K)), rng.standard_normal((M, K))
        W, W2 = rng.standard_normal((K, N)) * 0.05, rng.standard_normal((K, N)) * 0.05
        bias = rng.standard_normal(N).astype(np.float32)
        H = np.tanh(rng.standard_normal((M, N)))
        dA, dA2, dH = _bf16_dev(A, ldk), _bf16_dev(A2, ldk), _bf16_dev(H, N)
        Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        Bt2 = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        for w, bt in ((W, Bt), (W2, Bt2)):
            dw = _dev(w.astype(np.float32))
            call("mrl_pack_w_bf16", ctypes.c_void_p(dw.data_ptr()), K, N, 1, ctypes.c_void_p(bt.data_ptr()), ldk,
                 stream())
        db = _dev(bias)
        for out_bf in (0, 1):
            outs = []
            for big in ("0", "1", "1"):  # the tiled kernel, then the 256 x 256 kernel twice
                monkeypatch.setenv("MRL_GEMM_BIG_MIN_M", big)
                C = torch.full((M * N,), -7, dtype=torch.int16, device="cuda") if out_bf else \
                    torch.full((M * N,), float("nan"), dtype=torch.float32, device="cuda")
                g = _lib.GemmBf16Desc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=ldk,
                                      bt=ctypes.c_void_p(Bt.data_ptr()), ldb=ldk,
                                      a2=ctypes.c_void_p(dA2.data_ptr()) if dual else None,
                                      bt2=ctypes.c_void_p(Bt2.data_ptr()) if dual else None,
                                      c=ctypes.c_void_p(C.data_ptr()), ldc=N, c_bf16=out_bf, epilogue=E,
                                      bias=ctypes.c_void_p(db.data_ptr()), h=ctypes.c_void_p(dH.data_ptr()), ldh=N)
                call("mrl_gemm_bf16", ctypes.byref(g), None, stream())
                torch.cuda.synchronize()
                outs.append(C)
            assert torch.equal(outs[1], outs[2]), (M, N, K, dual, out_bf)
            diff = (outs[0] != outs[1]).sum().item()
            assert diff == 0, (M, N, K, dual, out_bf, diff,
                               (outs[0].float() - outs[1].float()).abs().max().item() if not out_bf else None)
            if not out_bf:
                f32_out = outs[1]
        rows = rng.choice(M, 300, replace=False)
        rows[0] = M - 1
        want = bfr(A[rows]) @ bfr(W)
        if dual:
            want = want + bfr(A2[rows]) @ bfr(W2)
        want = want + bias.astype(np.float64)
        if epi == "tanh":
            want = np.tanh(want)
        elif epi == "dtanh":
            hb = bfr(H[rows])
            want = want * (1.0 - hb * hb)
        got = f32_out.cpu().numpy().reshape(M, N)[rows].astype(np.float64)
        assert np.abs(got - want).max() / np.abs(want).max() < 2e-5, (M, N, K, dual)


def test_bf16_lds_limited_gemms_equal_default(monkeypatch):
    """The LDS-capped dispatch (desc.lds_limit > 0: the VF fit's GEMMs while they share CUs
    with the Humanoid rollout) takes only the non-persistent 128-row tiled kernels -- BK 64
    under an 80 KB cap, BK 32 under 64 KB -- and must write what the default dispatch (the
    persistent 256 x 256 kernels at these sizes) writes, bit for bit: NN single / dual,
    tanh / dtanh epilogues, f32 / bf16 outputs, row / K / N tails; TN slabs with the
    ones-row."""
    import ctypes

    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, stream
    rng = np.random.default_rng(21)
    monkeypatch.setenv("MRL_GEMM_STREAM_MIN_M", "0")
    for (M, N, K, ldk, dual, E) in [(70001, 512, 512, 512, True, _lib.GEMM_DTANH),
                                    (35000, 300, 377, 384, False, _lib.GEMM_TANH),
                                    (20000, 17, 512, 512, False, _lib.GEMM_STORE)]:
        A, A2 = rng.standard_normal((M, K)), rng.standard_normal((M, K))
        W, W2 = rng.standard_normal((K, N)) * 0.05, rng.standard_normal((K, N)) * 0.05
        bias = _dev(rng.standard_normal(N).astype(np.float32))
        dA, dA2, dH = _bf16_dev(A, ldk), _bf16_dev(A2, ldk), _bf16_dev(np.tanh(rng.standard_normal((M, N))), N)
        Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        Bt2 = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
        for w, bt in ((W, Bt), (W2, Bt2)):
            dw = _dev(w.astype(np.float32))
            call("mrl_pack_w_bf16", ctypes.c_void_p(dw.data_ptr()), K, N, 1, ctypes.c_void_p(bt.data_ptr()), ldk,
                 stream())
        for out_bf in (0, 1):
            outs = []
            for lim in (0, 81920, 65536):
                C = torch.full((M * N,), -7, dtype=torch.int16, device="cuda") if out_bf else \
                    torch.full((M * N,), float("nan"), dtype=torch.float32, device="cuda")
                g = _lib.GemmBf16Desc(m=M, n=N, k=K, a=ctypes.c_void_p(dA.data_ptr()), lda=ldk,
                                      bt=ctypes.c_void_p(Bt.data_ptr()), ldb=ldk,
                                      a2=ctypes.c_void_p(dA2.data_ptr()) if dual else None,
                                      bt2=ctypes.c_void_p(Bt2.data_ptr()) if dual else None,
                                      c=ctypes.c_void_p(C.data_ptr()), ldc=N, c_bf16=out_bf, epilogue=E,
                                      bias=ctypes.c_void_p(bias.data_ptr()), h=ctypes.c_void_p(dH.data_ptr()),
                                      ldh=N, lds_limit=lim)
                call("mrl_gemm_bf16", ctypes.byref(g), None, stream())
                torch.cuda.synchronize()
                outs.append(C)
            for i in (1, 2):
                assert torch.equal(outs[0], outs[i]), (M, N, K, dual, out_bf, i, (outs[0] != outs[i]).sum().item())
    for (R, din, dout, ones, splits) in [(40000, 512, 512, True, 64), (5000, 376, 300, True, 7)]:
        lda, ldb = (din + 7) // 8 * 8, (dout + 7) // 8 * 8
        dX, dG = _bf16_dev(rng.standard_normal((R, din)), lda), _bf16_dev(rng.standard_normal((R, dout)), ldb)
        Mr = din + (1 if ones else 0)
        S = int(_lib.load().mrl_gemm_slab_splits(R, splits))
        outs = []
        for lim in (0, 65536):
            slab = torch.full((S * Mr * dout,), float("nan"), dtype=torch.float32, device="cuda")
            g = _lib.GemmBf16TnDesc(m=Mr, n=dout, k=R, a=ctypes.c_void_p(dX.data_ptr()), lda=lda,
                                    b=ctypes.c_void_p(dG.data_ptr()), ldb=ldb, ones_row=int(ones), splits=splits,
                                    slab=ctypes.c_void_p(slab.data_ptr()), slab_stride=Mr * dout, ldc=dout,
                                    lds_limit=lim)
            call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())
            torch.cuda.synchronize()
            outs.append(slab.view(S, Mr, dout))
        # the rows above the ones-row: same per-slab k order in both kernels (the ones-row
        # differs in summation order between the 256 and 128 kernels, as tested above)
        assert torch.equal(outs[0][:, :din], outs[1][:, :din]), (R, din, dout)
