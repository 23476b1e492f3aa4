"""Multi-rank rehearsal of the data-parallel path with the real HIP kernels: two ranks
share the one GPU of the test box over torch.distributed gloo (the driver's 8-GPU run
uses RCCL with the same Comm calls).  Both ranks must take bit-identical steps."""
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
