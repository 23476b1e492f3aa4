"""The fp32 TRPO update at the benchmark's own size, against the float64 truth.

C3 (BASELINE configs[2]) runs the update over 4096 envs x 1024 steps = 4,194,304 Hopper
rows (11-64-64-3 DiagGauss policy).  The golden and oracle tests elsewhere use 400 to
70,001 rows; here the device path the headline runs -- split JVP rows + hybrid VJP in one launch,
per-wave slabs reduced over 4 M rows, device fp64 CG, batched line search -- is held to
the float64 oracle at north_star's 1e-4 on exactly that row count: the policy gradient
(`trpo.py:42-43`), one Fisher-vector product (`trpo.py:45-58`: the one-pass kernel, the
split pair and the exact-f32 pair) and a whole
`TrpoUpdater.__call__` (`trpo.py:72-140`: k exact; lm, shs, the step, the six stats).
The oracle is oracle/mlp_c.c (the numpy restatement's per-row math in C, pinned to it by
tests/test_oracle_c.py) driven by trpo_np.trpo_update, so the CG / line-search control
flow is the numpy oracle's own.  Run-to-run determinism of every Fisher-product kernel
is checked at the same size."""
import os
import time

import numpy as np
import pytest
import torch

from oracle import trpo_c as C
from oracle import trpo_np as T

pytestmark = pytest.mark.gpu
N = 4096 * 1024
THREADS = min(16, os.cpu_count() or 1)


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def batch():
    """A Hopper-shaped batch: fp32-representable obs / actions / advantages / oldprob,
    so device and oracle see identical inputs; oldprob = the policy's own rows (the
    rollout's), actions sampled from them, advantages correlated with the obs."""
    from modular_rl_amd import _lib
    from modular_rl_amd.core import DiagGauss, StochPolicyMLP
    from modular_rl_amd.nets import MlpNet
    t0 = time.time()
    rng = np.random.default_rng(2024)
    spec = T.Spec(11, [64, 64], 3, "gauss")
    th = T.mlp_init(rng, spec.shapes, True) + 0.1 * rng.standard_normal(spec.P)
    th[-3:] = -0.5 + 0.1 * rng.standard_normal(3)
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, 11), dtype=np.float32).astype(np.float64)
    net = MlpNet(11, 3, _lib.HEAD_GAUSS)
    net.set_flat(th)
    x = _dev(ob)
    # oldprob from the float64 forward of the oracle (chunked), rounded to fp32
    rows = T.RowChunks(ob, None, None, None, workers=THREADS, chunk=1 << 18)
    oldprob = np.concatenate(list(rows.pool.map(lambda s: T.policy_prob(spec, th, ob[s]), rows.sl)))
    oldprob = oldprob.astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, 3), dtype=np.float32)).astype(np.float32).astype(np.float64)
    adv = (rng.standard_normal(N, dtype=np.float32) + 0.5 * ob[:, 0]).astype(np.float64)
    adv = ((adv - adv.mean()) / adv.std()).astype(np.float32).astype(np.float64)
    crows = C.CRows(spec, ob, act, adv, oldprob, threads=THREADS)
    print(f"[fullsize] batch of {N} rows built in {time.time() - t0:.1f} s", flush=True)
    return dict(spec=spec, th=th, ob=ob, act=act, adv=adv, oldprob=oldprob, x=x, a=_dev(act), advd=_dev(adv),
                oldprobd=_dev(oldprob), crows=crows, pt=DiagGauss(3), net_cls=MlpNet)


def _net(b):
    from modular_rl_amd import _lib
    net = b["net_cls"](11, 3, _lib.HEAD_GAUSS)
    net.set_flat(b["th"])
    return net


@pytest.mark.parametrize("fisher", ["onepass", "split", "f32"])
def test_fullsize_gradient_and_fisher_product(batch, fisher, monkeypatch):
    """g and one Fisher product F v over all 4,194,304 rows, each within 1e-4 (max error
    relative to the vector's max) of the float64 oracle; every fp32 Fisher path (the
    default one-pass kernel, the split JVP rows + hybrid VJP pair, the exact-f32 pair); the
    one-pass case takes g from the one-launch policy gradient too."""
    monkeypatch.setenv("MRL_FISHER", "f32" if fisher == "f32" else "split")
    from modular_rl_amd import _lib
    b, spec = batch, batch["spec"]
    net = _net(b)
    assert net.fisher_split == (fisher != "f32")
    g = torch.zeros(net.P, device="cuda")
    if fisher == "onepass":  # the one-launch policy gradient (mrl_mlp_grad_hyb) records the cache
        assert net.policy_gradient(b["x"], N, 1.0 / N, b["a"], b["advd"], b["oldprobd"], g,
                                   torch.zeros(4, dtype=torch.float64, device="cuda"))
    else:
        gh = torch.zeros(N * net.gh, device="cuda")
        partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
        net.rows(_lib.EPI_SURRGRAD, b["x"], N, inv_n_global=1.0 / N, act=b["a"], adv=b["advd"],
                 oldprob=b["oldprobd"], ghead=gh, partial=partial)
        net.vjp_flat(b["x"], N, gh, g)
    t0 = time.time()
    g_want = b["crows"].pg(spec, b["th"])
    assert _rel(g.cpu().numpy().astype(np.float64), g_want) < 1e-4
    rng = np.random.default_rng(7)
    v = (rng.standard_normal(spec.P) * 0.05).astype(np.float32)
    vt = _dev(v)
    imgt = net.new_tangent_image()
    net.pack_tangent(vt, imgt)
    fv = torch.zeros(net.P, device="cuda")
    if fisher == "onepass":
        assert net.fisher_product(b["x"], N, 1.0 / N, vt, imgt, fv)
    else:
        fgh = torch.full((N * net.gh,), float("nan"), device="cuda")
        net.rows(_lib.EPI_FVP, b["x"], N, inv_n_global=1.0 / N, ghead=fgh, tangent=vt, image_t=imgt)
        net.vjp_flat(b["x"], N, fgh, fv)
    fv_want = b["crows"].fvp(spec, b["th"], v.astype(np.float64))
    print(f"[fullsize] oracle g + Fv in {time.time() - t0:.1f} s", flush=True)
    assert _rel(fv.cpu().numpy().astype(np.float64), fv_want) < 1e-4


_ORACLE_UPDATE = {}


@pytest.mark.parametrize("onepass", ["1", "0"])
def test_fullsize_trpo_update_matches_float64_oracle(batch, onepass, monkeypatch):
    """One whole TrpoUpdater.update at 4,194,304 rows (the bench's cg_damping 0.1,
    max_kl 0.01): accepted backtrack k exactly; lm, shs, the expected improve rate and
    the six loss stats within 1e-4 relative; theta within 1e-4 of the step -- with the
    one-pass Fisher product and policy gradient (default) and with the two-kernel pairs."""
    monkeypatch.setenv("MRL_FISHER_ONEPASS", onepass)
    monkeypatch.setenv("MRL_GRAD_ONEPASS", onepass)
    from modular_rl_amd.collector import Batch
    from modular_rl_amd.core import StochPolicyMLP
    from modular_rl_amd.trpo import TrpoUpdater
    b, spec = batch, batch["spec"]
    t0 = time.time()
    if not _ORACLE_UPDATE:
        _ORACLE_UPDATE["w"] = T.trpo_update(spec, b["th"], b["ob"], b["act"], b["adv"], b["oldprob"],
                                            cg_damping=0.1, max_kl=0.01, rows=b["crows"])
    th_w, stats_w, diag_w = _ORACLE_UPDATE["w"]
    print(f"[fullsize] oracle update in {time.time() - t0:.1f} s (k={diag_w['k']}, cg iters {diag_w['cg_iters']})",
          flush=True)
    pol = StochPolicyMLP(_net(b), b["pt"])
    assert pol.net.fisher_onepass == pol.net.grad_onepass == (onepass == "1")
    up = TrpoUpdater(pol, dict(cg_damping=0.1, max_kl=0.01))
    bt = Batch(N, b["x"], b["a"], b["oldprobd"])
    bt.adv = b["advd"]
    stats = up.update(bt)
    dg = up.last_diag
    assert dg["success"] and diag_w["success"]
    assert dg["k"] == diag_w["k"], (dg["k"], diag_w["k"])
    np.testing.assert_allclose([dg["lm"], dg["shs"], dg["expected_rate"]],
                               [diag_w["lm"], diag_w["shs"], diag_w["neggdotstepdir"] / diag_w["lm"]], rtol=1e-4)
    th1 = pol.get_flat().astype(np.float64)
    step = np.abs(th_w - b["th"]).max()
    assert np.abs(th1 - th_w).max() <= 1e-4 * step, np.abs(th1 - th_w).max() / step
    for k in stats_w:
        np.testing.assert_allclose(stats[k], stats_w[k], rtol=1e-4, atol=1e-7, err_msg=k)


def test_fullsize_onepass_policy_gradient_is_deterministic(batch):
    """The one-launch policy gradient (mrl_mlp_grad_hyb) repeated on the 4,194,304 rows:
    g, the loss sums and the activation cache it records, the same bits every time."""
    b = batch
    net = _net(b)
    assert net.grad_onepass
    outs = []
    for _ in range(3):
        g = torch.zeros(net.P, device="cuda")
        s = torch.zeros(4, dtype=torch.float64, device="cuda")
        assert net.policy_gradient(b["x"], N, 1.0 / N, b["a"], b["advd"], b["oldprobd"], g, s)
        outs.append((g, s))
        if len(outs) == 1:
            cache0 = net._cache(N).clone()
    assert torch.equal(net._cache(N), cache0)
    for g, s in outs[1:]:
        assert torch.equal(g, outs[0][0]) and torch.equal(s, outs[0][1])


@pytest.mark.parametrize("path", ["onepass", "split", "f32", "bf16"])
def test_fullsize_fisher_product_is_deterministic(batch, path, monkeypatch):
    """The Fisher product's kernels repeated on the same 4,194,304 rows give the same bits
    every time (the split JVP rows once did not: DESIGN §3, the packed-f32 hazard), for
    the one-pass kernel, the split pair, the exact-f32 pair and the bf16 pair."""
    monkeypatch.setenv("MRL_FISHER", "f32" if path == "f32" else "split")
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    b = batch
    net = MlpNet(11, 3, _lib.HEAD_GAUSS, dtype="bf16" if path == "bf16" else "fp32")
    net.set_flat(b["th"])
    gh = torch.zeros(N * net.gh, device="cuda")
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    net.rows(_lib.EPI_SURRGRAD, b["x"], N, inv_n_global=1.0 / N, act=b["a"], adv=b["advd"], oldprob=b["oldprobd"],
             ghead=gh, partial=partial)
    v = torch.randn(net.P, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3)) * 0.05
    imgt = net.new_tangent_image()
    net.pack_tangent(v, imgt)
    rows, fvs = [], []
    if path == "onepass":
        for _ in range(4):
            f = torch.zeros(net.P, device="cuda")
            assert net.fisher_product(b["x"], N, 1.0 / N, v, imgt, f)
            fvs.append(f)
        for f in fvs[1:]:
            assert torch.equal(f, fvs[0])
        return
    for _ in range(4):
        net.rows(_lib.EPI_FVP, b["x"], N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgt)
        rows.append(gh.clone())
        f = torch.zeros(net.P, device="cuda")
        net.vjp_flat(b["x"], N, gh, f)
        fvs.append(f)
    for r in rows[1:]:
        bad = (r != rows[0]).view(N, net.gh).any(dim=1).sum().item()
        assert bad == 0, f"{bad} rows differ"
    for f in fvs[1:]:
        assert torch.equal(f, fvs[0])
