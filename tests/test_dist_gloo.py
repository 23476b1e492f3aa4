"""Data-parallel orchestration on CPU with torch.distributed gloo, world_size 2.

* TrpoUpdater.update with the rows split over 2 ranks takes the same step as one
  rank holding all rows, and as the float64 oracle (the collectives are placed and
  scaled correctly: g, every CG Fvp, loss sums, line-search losses).
* merge_filter_deltas: 2 ranks pushing different observations from a common start
  end with the running stat of one process pushing all of them (rank order).
* vf.LbfgsOptimizer (the VF fit, `core.py:663-697`) with the rows split over 2 ranks
  (loss sums and gradients all-reduced per L-BFGS evaluation, scaled by 1/N_global)
  ends where one rank holding all rows does, and where scipy L-BFGS-B on the float64
  oracle loss does -- also with its reductions over a host (gloo) group (Comm.host,
  what the pipelined loop uses while the fit overlaps the rollout at world > 1).
"""
import os
import types

import numpy as np
import pytest
import scipy.optimize
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import trpo_np as T


def _data(seed=0, N=600):
    rng = np.random.default_rng(seed)
    spec = T.Spec(11, [64, 64], 3, "gauss")
    th = T.mlp_init(rng, spec.shapes, True) + 0.02 * rng.standard_normal(spec.P)
    ob = rng.standard_normal((N, 11))
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob)
    act = T.sample(spec, oldprob, rng.standard_normal((N, 3)))
    adv = T.standardize(rng.standard_normal(N) + 0.4 * ob[:, 1])
    return spec, th, ob, act, adv, oldprob


def _update(rank_rows, comm):
    from modular_rl_amd.trpo import TrpoUpdater
    from tests.oracle_ops import OracleOps, fake_policy
    spec, th, ob, act, adv, oldprob = _data()
    sl = rank_rows
    pol = fake_policy(spec, th)
    up = TrpoUpdater(pol, dict(cg_damping=0.1, max_kl=0.01), comm=comm, ops=OracleOps(spec, pol.net))
    b = types.SimpleNamespace(n=len(ob[sl]), obs=ob[sl], act=act[sl], adv=adv[sl], prob=oldprob[sl])
    stats = up.update(b)
    return pol.net.theta.numpy().copy(), stats, up.last_diag


def _vf_data(N=600):
    rng = np.random.default_rng(7)
    spec = T.Spec(6, [64, 64], 1, "linear")
    th = (T.mlp_init(rng, spec.shapes, False) + 0.05 * rng.standard_normal(spec.P)).astype(np.float32)
    X = rng.standard_normal((N, 6)).astype(np.float32).astype(np.float64)
    y = (np.sin(X[:, 0]) + 0.5 * X[:, 1] * X[:, 2] + 0.1 * rng.standard_normal(N)).astype(np.float32)
    return spec, th, X, y


def _vf_fit(rank_rows, comm):
    from modular_rl_amd.vf import LbfgsOptimizer
    from tests.oracle_ops import OracleVfNet
    spec, th, X, y = _vf_data()
    net = OracleVfNet(spec, th)
    opt = LbfgsOptimizer(net, maxiter=2, comm=comm)
    x, t = X[rank_rows], torch.as_tensor(y[rank_rows], dtype=torch.float64)
    n_glob = comm.allreduce_int(len(x))
    info = opt.update((x, None, 1.0, len(x), t, n_glob))
    return net.get_flat().astype(np.float64), info


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from modular_rl_amd.collector import merge_filter_deltas
    from modular_rl_amd.dist import Comm
    comm = Comm()
    N = 600
    rows = slice(rank * N // world, (rank + 1) * N // world)
    th, stats, diag = _update(rows, comm)
    # filter merge: common start state (from pushes of `pre`), then rank-local pushes
    rng = np.random.default_rng(1)
    pre = rng.standard_normal((30, 4)) * 2 + 1
    local = [rng.standard_normal((17 + 5 * r, 4)) * (r + 1) for r in range(world)]
    lrew = [rng.standard_normal(17 + 5 * r) for r in range(world)]
    rs, rr = T.RunningStat((4,)), T.RunningStat(())
    for x in pre:
        rs.push(x)
        rr.push(x[0])
    s0 = np.concatenate([[rs.n, rr.n], np.append(rs.M, rr.M), np.append(rs.S, rr.S)])
    for x, r in zip(local[rank], lrew[rank]):
        rs.push(x)
        rr.push(r)
    s1 = np.concatenate([[rs.n, rr.n], np.append(rs.M, rr.M), np.append(rs.S, rr.S)])
    merged = merge_filter_deltas(s0, s1, comm)
    th_vf, info_vf = _vf_fit(rows, comm)
    # the fit's reductions over a host group (Comm.host: what the pipelined loop uses
    # while the fit overlaps the rollout in data-parallel mode) take the same path
    from modular_rl_amd.core import fit_comm_for
    from modular_rl_amd.dist import HostComm
    hcomm = Comm(host_group=dist.new_group(backend="gloo"))
    fc = fit_comm_for(hcomm, True)
    assert isinstance(fc, HostComm) and fit_comm_for(hcomm, False) is hcomm
    th_vf_h, info_vf_h = _vf_fit(rows, fc)
    if rank == 0:
        q.put((th, dict(stats), diag["k"], merged, th_vf, dict(info_vf), th_vf_h, dict(info_vf_h)))
    dist.destroy_process_group()


def _get(q, procs, timeout):
    """q.get that fails as soon as a rank has died instead of waiting out the timeout."""
    import queue
    import time
    end = time.time() + timeout
    while time.time() < end:
        try:
            return q.get(timeout=2)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, "rank exited with %s" % dead
    raise AssertionError("no result within %ss" % timeout)


def test_two_rank_update_equals_single_rank_and_oracle():
    from modular_rl_amd.dist import Comm
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    th2, stats2, k2, merged, thv2, infov2, thv2h, infov2h = _get(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    th1, stats1, diag1 = _update(slice(0, 600), Comm())
    spec, th, ob, act, adv, oldprob = _data()
    th_w, stats_w, diag_w = T.trpo_update(spec, th, ob, act, adv, oldprob, cg_damping=0.1, max_kl=0.01)
    step = np.abs(th_w - th).max()
    assert np.abs(th2 - th1).max() <= 1e-9 * step
    assert np.abs(th1 - th_w).max() <= 1e-9 * step
    assert k2 == diag1["k"] == diag_w["k"]
    for k in stats_w:
        np.testing.assert_allclose(stats2[k], stats_w[k], rtol=1e-9, atol=1e-13)
    # filter: all pushes in rank order from the common start
    rng = np.random.default_rng(1)
    pre = rng.standard_normal((30, 4)) * 2 + 1
    local = [rng.standard_normal((17 + 5 * r, 4)) * (r + 1) for r in range(2)]
    lrew = [rng.standard_normal(17 + 5 * r) for r in range(2)]
    rs, rr = T.RunningStat((4,)), T.RunningStat(())
    for x in pre:
        rs.push(x)
        rr.push(x[0])
    for r in range(2):
        for x, rw in zip(local[r], lrew[r]):
            rs.push(x)
            rr.push(rw)
    want = np.concatenate([[rs.n, rr.n], np.append(rs.M, rr.M), np.append(rs.S, rr.S)])
    np.testing.assert_allclose(merged, want, rtol=1e-10, atol=1e-10)
    # VF fit: 2 ranks == 1 rank (float32 gradients summed per rank) == scipy on the oracle
    thv1, infov1 = _vf_fit(slice(0, 600), Comm())
    spec, thv, X, y = _vf_data()

    def lossandgrad(t):
        l, g, _, _ = T.vf_loss_grad(spec, t.astype(np.float32).astype(np.float64), X, y.astype(np.float64))
        return float(l), g

    thw, _, _ = scipy.optimize.fmin_l_bfgs_b(lossandgrad, thv.astype(np.float64), maxiter=2)
    move = np.abs(thw - thv).max()
    assert move > 1e-3
    assert np.abs(thv2 - thv1).max() <= 1e-4 * move
    assert np.abs(thv1 - thw.astype(np.float32)).max() <= 1e-5 * move
    for k in ("loss_before", "loss_after", "mse_before", "mse_after"):
        np.testing.assert_allclose(infov2[k], infov1[k], rtol=1e-6)
    # host-group reductions: the same sums, the same fit
    np.testing.assert_array_equal(thv2h, thv2)
    assert infov2h == infov2
    assert infov1["loss_after"] < infov1["loss_before"]
