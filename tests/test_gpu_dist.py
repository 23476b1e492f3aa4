"""Multi-rank rehearsal of the data-parallel path with the real HIP kernels: two ranks
share the one GPU of the test box over torch.distributed gloo (the driver's 8-GPU run
uses RCCL with the same Comm calls).  Both ranks must take bit-identical steps, and a
2-rank TrpoUpdater.update on two halves of a fixed batch must equal the 1-rank HIP
update on the union batch (`trpo.py:72-140`: g and every CG Fvp summed over ranks).
Unmeasured on hardware at world > 1 with RCCL (the pool's boxes have one GPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, env_id, agent_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MRL_DIST_BACKEND="gloo")
    from modular_rl_amd import agentzoo
    from modular_rl_amd.core import run_policy_gradient_algorithm
    from modular_rl_amd.dist import init_from_env
    from modular_rl_amd.envs import make
    comm = init_from_env()
    env = make(env_id)
    cfg = dict(n_envs=64, horizon=32, timestep_limit=env.spec.max_episode_steps, n_iter=2, gamma=0.995, lam=0.97,
               max_kl=0.01, cg_damping=0.1, maxiter=3, epochs=1, timesteps_per_batch=64 * 32, use_graph=1)
    if env_id == "Humanoid-v2":
        cfg["hid_sizes"] = [128, 128]
    agent = getattr(agentzoo, agent_name)(env.observation_space, env.action_space, cfg, comm=comm)
    seen = []
    run_policy_gradient_algorithm(env, agent, callback=lambda st: seen.append(dict(st)), usercfg=cfg)
    col = agent._filter_owner()
    q.put((rank, agent.policy.get_flat(), agent.baseline.net.get_flat(), col.filter_state[:col.FS].cpu().numpy(),
           [{k: float(v) for k, v in st.items() if np.asarray(v).size == 1} for st in seen]))


@pytest.mark.parametrize("env_id,agent_name", [("Hopper-v2", "TrpoAgent"), ("CartPole-v0", "PpoLbfgsAgent"),
                                               ("Humanoid-v2", "TrpoAgent")])
def test_two_ranks_take_identical_steps(env_id, agent_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, env_id, agent_name, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=600) for _ in procs], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, th0, vf0, fs0, st0), (_, th1, vf1, fs1, st1) = out
    assert np.array_equal(th0, th1) and np.array_equal(vf0, vf1)
    assert np.array_equal(fs0, fs1)
    assert len(st0) == 2 and st0[-1]["pol_kl_after"] == st1[-1]["pol_kl_after"]
    # the ranks' batches differ (env ids rank*E ..), the global episode stats agree
    assert st0[-1]["EpRewMean"] == st1[-1]["EpRewMean"]


def _split_batch(seed=11, N=16384):
    """A fixed Hopper-shaped batch (fp32-representable) and the policy's theta."""
    from oracle import trpo_np as T
    rng = np.random.default_rng(seed)
    spec = T.Spec(11, [64, 64], 3, "gauss")
    th = T.mlp_init(rng, spec.shapes, True) + 0.05 * rng.standard_normal(spec.P)
    th[-3:] = -0.5
    th = th.astype(np.float32).astype(np.float64)
    ob = rng.standard_normal((N, 11)).astype(np.float32)
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob.astype(np.float64)).astype(np.float32)
    act = T.sample(spec, oldprob.astype(np.float64), rng.standard_normal((N, 3))).astype(np.float32)
    adv = T.standardize(rng.standard_normal(N) + 0.4 * ob[:, 1]).astype(np.float32)
    return th, ob, act, adv, oldprob


def _hip_update(rows, comm, n_global):
    import torch
    from modular_rl_amd import _lib
    from modular_rl_amd.collector import Batch
    from modular_rl_amd.core import DiagGauss, StochPolicyMLP
    from modular_rl_amd.nets import MlpNet
    from modular_rl_amd.trpo import TrpoUpdater
    th, ob, act, adv, oldprob = _split_batch()
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a[rows])).cuda()
    net = MlpNet(11, 3, _lib.HEAD_GAUSS)
    net.set_flat(th)
    pol = StochPolicyMLP(net, DiagGauss(3))
    up = TrpoUpdater(pol, dict(cg_damping=0.1, max_kl=0.01), comm=comm)
    b = Batch(len(ob[rows]), dev(ob), dev(act), dev(oldprob))
    b.adv = dev(adv)
    b.n_global = n_global
    stats = up.update(b)
    d = up.last_diag
    return pol.get_flat().astype(np.float64), {k: float(v) for k, v in stats.items()}, \
        dict(k=d["k"], lm=d["lm"], shs=d["shs"], rate=d["expected_rate"])


def _split_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MRL_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from modular_rl_amd.dist import Comm, init_from_env
    comm = init_from_env()
    assert comm.enabled and comm.world == world
    N = 16384
    two = _hip_update(slice(rank * N // world, (rank + 1) * N // world), comm, N)
    dist.barrier()
    dist.destroy_process_group()
    one = _hip_update(slice(0, N), Comm(), N) if rank == 0 else None
    q.put((rank, two, one))


def test_two_rank_update_equals_one_rank_union_batch():
    """2 gloo ranks on one GPU, each updating on half of a fixed 16,384-row batch (filter
    frozen: the batch is given), against the 1-rank HIP update on the whole batch: theta
    within 1e-6 of the step, k exact, lm / shs / rate and the six stats within 1e-6
    relative (the ranks' slab sums are added in another order, so bits may differ)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=600) for _ in procs], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, (th0, st0, d0), (th1, st1, d1)), (_, (th0b, st0b, d0b), _) = out
    assert np.array_equal(th0, th0b) and d0 == d0b  # the two ranks agree bit for bit
    step = np.abs(th1 - _split_batch()[0]).max()
    assert step > 0
    err = np.abs(th0 - th1).max() / step
    print(f"[dp2] theta rel-to-step {err:.2e}, k {d0['k']} / {d1['k']}", flush=True)
    assert d0["k"] == d1["k"]
    assert err <= 1e-6, err
    np.testing.assert_allclose([d0["lm"], d0["shs"], d0["rate"]], [d1["lm"], d1["shs"], d1["rate"]], rtol=1e-6)
    for k in st1:
        np.testing.assert_allclose(st0[k], st1[k], rtol=1e-6, atol=1e-9, err_msg=k)
