"""The pipelined iteration loop (VF fit of iteration k on a CU-masked stream beside
the rollout of iteration k+1) against the reference order: every parameter, filter
statistic and reported stat is bit-identical."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(env_id, pipeline, n_iter=3, agent_cls="TrpoAgent", prelaunch=False, **kw):
    from modular_rl_amd import agentzoo
    from modular_rl_amd.core import IterationRunner
    from modular_rl_amd.envs import make
    env = make(env_id)
    cfg = dict(timestep_limit=env.spec.max_episode_steps, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1,
               n_envs=256, horizon=64, seed=3, use_graph=1)
    cfg.update(kw)
    agent = getattr(agentzoo, agent_cls)(env.observation_space, env.action_space, cfg)
    col = agent.make_collector(env, cfg)
    runner = IterationRunner(agent, col, cfg, pipeline=pipeline)
    runner.record_phases = True  # the phase events (off by default outside timed measurements)
    stats = []
    with runner.loop_stream():
        for i in range(n_iter):
            s = runner.step(prelaunch_next=prelaunch and i + 1 < n_iter)
            if s is not None:
                stats.append(s)
        s = runner.drain()
    if s is not None:
        stats.append(s)
    torch.cuda.synchronize()
    return runner, agent, col, stats


@pytest.mark.parametrize("env_id,agent_cls,kw", [("Hopper-v2", "TrpoAgent", {}), ("CartPole-v0", "TrpoAgent", {}),
                                                 ("Hopper-v2", "PpoLbfgsAgent", {}),
                                                 ("Humanoid-v2", "TrpoAgent", dict(n_envs=128, horizon=16,
                                                                                   hid_sizes=[128, 96]))])
@pytest.mark.parametrize("prelaunch", [False, True])
def test_pipelined_loop_is_bit_identical(env_id, agent_cls, kw, prelaunch):
    """...and with the next rollout issued from the update (prelaunch: as soon as theta is
    final, before the stats / capture / loop Python), in both orders."""
    r0, a0, c0, s0 = _run(env_id, False, agent_cls=agent_cls, **kw)
    r1, a1, c1, s1 = _run(env_id, True, agent_cls=agent_cls, prelaunch=prelaunch, **kw)
    assert not r0.pipeline and r1.pipeline  # few rollout blocks: the CU split applies
    assert len(s0) == len(s1) == 3
    np.testing.assert_array_equal(a0.policy.net.get_flat(), a1.policy.net.get_flat())
    np.testing.assert_array_equal(a0.baseline.net.get_flat(), a1.baseline.net.get_flat())
    np.testing.assert_array_equal(c0.filter_state.cpu().numpy(), c1.filter_state.cpu().numpy())
    for x, y in zip(s0, s1):
        assert list(x) == list(y)
        for k in x:
            assert x[k] == y[k] or (np.isnan(x[k]) and np.isnan(y[k])), k


def test_masked_streams_are_disjoint():
    from modular_rl_amd import streams
    from modular_rl_amd.core import rollout_cu_split
    n = streams.cu_count()
    rc, vc = rollout_cu_split(64, n)
    R, V = streams.masked_stream(rc), streams.masked_stream(vc)
    assert streams.stream_cus(R) == rc and streams.stream_cus(V) == vc
    assert rollout_cu_split(n, n) is None


@pytest.mark.parametrize("pipeline", [False, True])
def test_prelaunched_rollout_is_bit_identical(pipeline):
    """Hopper, TRPO: the loop with every next rollout issued from the update equals the
    plain loop bit for bit (parameters, filter, every reported stat)."""
    r0, a0, c0, s0 = _run("Hopper-v2", pipeline, n_iter=4)
    r1, a1, c1, s1 = _run("Hopper-v2", pipeline, n_iter=4, prelaunch=True)
    np.testing.assert_array_equal(a0.policy.net.get_flat(), a1.policy.net.get_flat())
    np.testing.assert_array_equal(a0.baseline.net.get_flat(), a1.baseline.net.get_flat())
    np.testing.assert_array_equal(c0.filter_state.cpu().numpy(), c1.filter_state.cpu().numpy())
    assert len(s0) == len(s1) == 4
    for x, y in zip(s0, s1):
        for k in x:
            assert x[k] == y[k] or (np.isnan(x[k]) and np.isnan(y[k])), k


@pytest.mark.parametrize("lds,wpb", [("0", "1"), ("65536", "4")])
def test_cosched_fit_beside_wave_per_env_rollout_is_bit_identical(lds, wpb, monkeypatch):
    """C5's per-GPU width (1024 Humanoid envs: the wave-per-env step wants E / 4 = 256 CUs,
    so no disjoint CU split): with MRL_COSCHED_FIT=1 the VF fit of iteration k shares the
    CUs with the rollout of k+1 on two plain streams, bit-identical to the reference order;
    also with the fit's GEMMs capped at 64 KB of LDS and four-env Humanoid blocks."""
    monkeypatch.setenv("MRL_COSCHED_FIT", "1")
    monkeypatch.setenv("MRL_COSCHED_LDS", lds)
    monkeypatch.setenv("MRL_HM_WPB", wpb)
    kw = dict(n_envs=1024, horizon=8, hid_sizes=[64, 64])
    r0, a0, c0, s0 = _run("Humanoid-v2", False, **kw)
    r1, a1, c1, s1 = _run("Humanoid-v2", True, prelaunch=True, **kw)
    assert not r0.pipeline and r1.pipeline
    np.testing.assert_array_equal(a0.policy.net.get_flat(), a1.policy.net.get_flat())
    np.testing.assert_array_equal(a0.baseline.net.get_flat(), a1.baseline.net.get_flat())
    np.testing.assert_array_equal(c0.filter_state.cpu().numpy(), c1.filter_state.cpu().numpy())
    assert len(s0) == len(s1) == 3
    for x, y in zip(s0, s1):
        for k in x:
            assert x[k] == y[k] or (np.isnan(x[k]) and np.isnan(y[k])), k


def test_fit_runs_beside_the_prelaunched_rollout():
    """With the next rollout issued from the update, the deferred VF fit of the previous
    iteration still starts while that rollout runs (loop_stream: no legacy-stream event
    that would wait for the CU-masked rollout stream): its first event precedes the
    rollout's end event on the device timeline."""
    runner, agent, col, stats = _run("Hopper-v2", True, n_iter=3, prelaunch=True, n_envs=256, horizon=1024)
    ev = runner.last_phase_events
    assert "vf0" in ev and "rollout1" in ev
    assert ev["vf0"].elapsed_time(ev["rollout1"]) > 0.5  # ms of the rollout left when the fit began


def test_value_order_sequences_two_streams():
    """streams.ValueOrder (the pipelined loop's rollout <-> iteration ordering on a memory
    value): a ping-pong of dependent read-modify-writes between a CU-masked stream and a
    plain one, each hop behind a long kernel on the producer, ends with every update
    applied in order (x = 2 N), as an event-ordered ping-pong does."""
    from modular_rl_amd import streams
    n_cu = streams.cu_count()
    a = streams.masked_stream(list(range(min(64, n_cu))))
    b = torch.cuda.Stream()
    order = streams.ValueOrder()
    x = torch.zeros(1 << 20, device="cuda")
    N = 50
    for i in range(N):
        with torch.cuda.stream(a):
            torch.cuda._sleep(20000)  # the producer's work finishes after the host enqueued the wait
            x.mul_(1.0).add_(1.0)
        order.order(a, b)
        with torch.cuda.stream(b):
            x.add_(1.0)
        order.order(b, a)
    torch.cuda.synchronize()
    assert torch.all(x == 2 * N)
