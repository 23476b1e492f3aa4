"""The RCCL path on one GPU, and the persistent rollout's abort made visible.

* RCCL: ``torch.distributed`` with backend ``nccl`` (RCCL on ROCm) at world size 1
  and the communicator forced on (``MRL_COMM_FORCE=1``), so every all-reduce /
  all-gather of the data-parallel design (g, each CG Fisher product, loss sums,
  advantage moments, VF loss + gradient, episode stats, the filter merge) runs
  through RCCL on the pipelined loop's streams -- the RCCL kernels share the device
  with the CU-masked rollout stream (persistent launch) and the fit stream.  A sum
  over one rank is the identity, so parameters, VF parameters, filter state and every
  reported stat must equal the run without a communicator bit for bit.  (The reference
  has no data-parallel path: ``parallel`` raises NotImplementedError, core.py:123-124;
  the per-Fvp reduction follows trpo.py:86-92.)
* Abort: a persistent rollout whose grid cannot be resident gives up (bounded polls)
  and leaves its trajectories incomplete; the iteration must raise MrlError instead
  of training on them (core.py:182-207 requires whole trajectories)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _train(env_id, agent_name, comm):
    from modular_rl_amd import agentzoo
    from modular_rl_amd.core import run_policy_gradient_algorithm
    from modular_rl_amd.envs import make
    env = make(env_id)
    cfg = dict(n_envs=4096, horizon=24, timestep_limit=env.spec.max_episode_steps, n_iter=2, gamma=0.995, lam=0.97,
               max_kl=0.01, cg_damping=0.1, timesteps_per_batch=4096 * 24, use_graph=1, pipeline=1, seed=5)
    agent = getattr(agentzoo, agent_name)(env.observation_space, env.action_space, cfg, comm=comm)
    seen = []
    run_policy_gradient_algorithm(env, agent, callback=lambda st: seen.append(dict(st)), usercfg=cfg)
    torch.cuda.synchronize()
    col = agent._filter_owner()
    return (agent.policy.get_flat(), agent.baseline.net.get_flat(), col.filter_state[:col.FS].cpu().numpy(),
            [{k: float(v) for k, v in st.items() if np.asarray(v).size == 1 and k != "TimeElapsed"} for st in seen],
            col.persistent and not col.layered)


def _worker(port, cases, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        from modular_rl_amd.dist import Comm, init_from_env
        plain = [_train(e, a, Comm()) for e, a in cases]
        os.environ["MRL_COMM_FORCE"] = "1"
        comm = init_from_env()
        backend = torch.distributed.get_backend()
        assert comm.enabled and comm.world == 1
        rccl = [_train(e, a, comm) for e, a in cases]
        torch.distributed.destroy_process_group()
        q.put(("ok", backend, plain, rccl))
    except BaseException as ex:  # report, do not hang the parent
        import traceback
        q.put(("error", repr(ex), traceback.format_exc(), None))


def test_rccl_world1_forced_comm_is_bit_identical():
    cases = [("Hopper-v2", "TrpoAgent"), ("CartPole-v0", "PpoLbfgsAgent")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), cases, q))
    p.start()
    out = q.get(timeout=400)
    p.join(timeout=60)
    assert out[0] == "ok", out[2]
    _, backend, plain, rccl = out
    assert backend == "nccl"
    assert p.exitcode == 0
    for (case, a, b) in zip(cases, plain, rccl):
        th0, vf0, fs0, st0, persistent = a
        th1, vf1, fs1, st1, _ = b
        assert persistent, case  # the persistent rollout ran beside the RCCL kernels
        np.testing.assert_array_equal(th0, th1, err_msg=str(case))
        np.testing.assert_array_equal(vf0, vf1, err_msg=str(case))
        np.testing.assert_array_equal(fs0, fs1, err_msg=str(case))
        assert len(st0) == len(st1) == 2
        for x, y in zip(st0, st1):
            assert list(x) == list(y)
            for k in x:
                assert x[k] == y[k] or (np.isnan(x[k]) and np.isnan(y[k])), (case, k)


# ------------------------------------------------------------------ abort path
def _runner(pipeline, agent_cls="TrpoAgent"):
    from modular_rl_amd import agentzoo
    from modular_rl_amd.core import IterationRunner
    from modular_rl_amd.envs import make
    env = make("Hopper-v2")
    cfg = dict(timestep_limit=1000, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1, n_envs=4096, horizon=4,
               seed=3, use_graph=0)
    agent = getattr(agentzoo, agent_cls)(env.observation_space, env.action_space, cfg)
    col = agent.make_collector(env, cfg)
    return IterationRunner(agent, col, cfg, pipeline=pipeline), col


def test_rollout_on_too_few_cus_falls_back_to_step_launches():
    """The residency check counts the CUs of the stream the rollout runs on: 64 blocks
    on a 2-CU stream run as step launches, complete, with no abort."""
    from modular_rl_amd import streams
    runner, col = _runner(pipeline=False)
    with torch.cuda.stream(streams.masked_stream([0, 1])):
        st = runner.step()
    torch.cuda.synchronize()
    assert st is not None and col.desc.launch_cus == 2
    col.check()


@pytest.mark.parametrize("pipeline,agent_cls", [(False, "TrpoAgent"), (True, "TrpoAgent"),
                                                (False, "PpoLbfgsAgent"), (True, "PpoSgdAgent")])
def test_persistent_abort_raises_in_the_iteration(pipeline, agent_cls):
    """64 persistent blocks forced onto 2 CUs (debug flag past the residency check):
    the resident blocks give up after their bounded polls, the rest exit on the abort
    word, and IterationRunner.step() raises MrlError instead of reporting the
    iteration: the policy update reads the status back with its step scalars (TRPO) or
    checks it first (Batch.check_abort, both PPO updaters) and raises before it touches
    theta."""
    from modular_rl_amd import streams
    from modular_rl_amd._lib import MrlError
    runner, col = _runner(pipeline=pipeline, agent_cls=agent_cls)
    col.force_persistent = True
    two = streams.masked_stream([0, 1])
    theta0 = runner.agent.policy.net.theta.clone()
    with pytest.raises(MrlError, match="resident"):
        if pipeline:
            assert runner.pipeline
            runner.rollout_stream = two
            for _ in range(3):
                runner.step()
        else:
            with torch.cuda.stream(two):
                runner.step()
    torch.cuda.synchronize()
    assert int(col.status.item()) != 0
    # the update read the abort status back with its step scalars: the policy never
    # consumed the incomplete trajectories
    assert torch.equal(runner.agent.policy.net.theta, theta0)
    with pytest.raises(MrlError, match="resident"):
        col.check()
