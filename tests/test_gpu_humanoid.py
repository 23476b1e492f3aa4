"""GPU parity of the layered-policy rollout (mrl_rollout_obs / GEMM forward /
mrl_rollout_act) and of the Humanoid config (376-512-512-512-17)
against the float64 oracle, plus an end-to-end Humanoid TRPO iteration."""
import numpy as np
import pytest
import torch

from oracle import rollout_np as RO
from oracle import trpo_np as T

pytestmark = pytest.mark.gpu


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def _layered_policy(head, nin, nout, hid, seed, logstd0=-0.5):
    from modular_rl_amd import _lib
    from modular_rl_amd.core import Categorical, DiagGauss, StochPolicyMLP
    from modular_rl_amd.nets import LayeredMlpNet
    rng = np.random.default_rng(seed)
    spec = T.Spec(nin, hid, nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.02 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = logstd0 + 0.1 * rng.standard_normal(nout)
    th = th.astype(np.float32).astype(np.float64)
    net = LayeredMlpNet(nin, nout, _lib.HEAD_GAUSS if head == "gauss" else _lib.HEAD_SOFTMAX, hid)
    net.set_flat(th)
    pt = DiagGauss(nout) if head == "gauss" else Categorical(nout)
    return spec, th, StochPolicyMLP(net, pt)


KINDS = {"CartPole-v0": RO.CARTPOLE, "Hopper-v2": RO.HOPPER, "Humanoid-v2": RO.HUMANOID}


@pytest.mark.parametrize("env_id,hid,E,Tn,limit,inject", [
    ("Hopper-v2", [64, 64], 150, 24, 1000, False),
    ("CartPole-v0", [32], 7, 30, 12, True),
    ("Humanoid-v2", [512, 512, 512], 40, 12, 1000, False),
    ("Humanoid-v2", [128, 64], 130, 10, 6, True),
    # articulated Humanoid-v2: ~22-step episodes under this policy end (healthy-z
    # test) and auto-reset inside the horizon
    ("Humanoid-v2", [64, 64], 64, 60, 1000, False),
])
def test_layered_rollout_matches_oracle(env_id, hid, E, Tn, limit, inject):
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.envs import make
    env = make(env_id)
    head = "softmax" if env.discrete else "gauss"
    spec, th, pol = _layered_policy(head, env.obs_dim, env.act_dim, hid, seed=E)
    seed = 777 + E
    col = Collector(env, pol, E, Tn, limit, filter=1, seed=seed, use_graph=False)
    assert col.layered
    envs = RO.Envs(KINDS[env_id], E, seed)
    fs = RO.FilterState(env.obs_dim + 1)
    for it in range(2):
        noise = None
        if inject:
            rng = np.random.default_rng(it)
            noise = rng.random((Tn, E)) if env.discrete else rng.standard_normal((Tn, E, env.act_dim))
            col.set_noise(noise.reshape(Tn * E, -1) if not env.discrete else noise.reshape(-1))
        b = col.collect()
        want, fs = RO.collect(envs, fs, spec, th, Tn, limit, it, filt=True, noise=noise)
        if env_id == "Humanoid-v2" and Tn >= 60:
            assert (want["flags"] & 2).any()  # terminations happened (and were reset)
        np.testing.assert_array_equal(b.flags.cpu().numpy().reshape(Tn, E), want["flags"])
        np.testing.assert_array_equal(b.ep_t.cpu().numpy().reshape(Tn, E), want["ep_t"])
        np.testing.assert_allclose(b.obs.cpu().numpy().reshape(Tn, E, -1), want["obs"], rtol=1e-4, atol=1e-4)
        if env.discrete:
            np.testing.assert_array_equal(b.act.cpu().numpy().reshape(Tn, E), want["act"])
        else:
            np.testing.assert_allclose(b.act.cpu().numpy().reshape(Tn, E, -1), want["act"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(b.prob.cpu().numpy().reshape(Tn, E, -1), want["prob"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(b.rew.cpu().numpy().reshape(Tn, E), want["rew"], rtol=1e-4, atol=1e-3)
        (n, m, var), (nr, mr, vr) = col.filter_stats()
        assert n == fs.n and nr == fs.nr
        np.testing.assert_allclose(m, fs.M[:-1], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(mr, fs.M[-1], rtol=1e-4, atol=1e-5)


def test_humanoid_step_matches_oracle_twin():
    """The wave-per-env Humanoid step (hm_act_kernel) against oracle/humanoid.py on the
    same controls: with the policy means given as z rows, logstd 0 and injected noise the
    action a = z + noise is the same fp32 value on both sides, and the fp64 env state
    (qpos ++ qvel ++ ctrl) and the raw 376-d observation + reward after every one of 40
    steps (auto-resets included) follow the oracle's operation sequence per value.  Not
    bit for bit: the device sin / cos and numpy's libm differ in the last bit for some
    angles (about half the words differ after 40 steps, by <= ~1e-9 relative, r06s2d).
    Bit-identity of a kernel change against the previous build is tools/hm_twin_ab.py."""
    from modular_rl_amd import _lib
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.envs import make
    from modular_rl_amd._lib import call, ptr, stream
    import ctypes
    env = make("Humanoid-v2")
    E, Tn, A, O = 96, 40, env.act_dim, env.obs_dim
    _, _, pol = _layered_policy("gauss", O, A, [32], seed=4)
    seed = 4242
    col = Collector(env, pol, E, Tn, 1000, filter=1, seed=seed, use_graph=False)
    rng = np.random.default_rng(11)
    noise = rng.standard_normal((Tn, E, A))
    z = (0.4 * rng.standard_normal((Tn, E, A))).astype(np.float32)
    col.set_noise(noise.reshape(Tn * E, A))
    logstd = torch.zeros(A, dtype=torch.float32, device="cuda")
    d, bufs = ctypes.byref(col.desc), col._bufs()
    envs = RO.Envs(RO.HUMANOID, E, seed)
    envs.reset(np.arange(E))
    call("mrl_rollout_reset_rows", d, ctypes.byref(bufs), stream())
    ns = envs.ns

    worst = [0.0, 0, 0]  # max relative difference, differing words, compared words

    def cmp(got, want):
        worst[1] += int((got.view(np.uint64) != want.view(np.uint64)).sum())
        worst[2] += got.size
        worst[0] = max(worst[0], float((np.abs(got - want) / np.maximum(np.abs(want), 1e-6)).max()))

    def check(t, rew=None):
        torch.cuda.synchronize()
        cmp(col.env_state[:ns * E].view(ns, E).cpu().numpy().T, envs.state)
        raw = col.raw_obs.view(O + 1, E).cpu().numpy().T
        cmp(raw[:, :O], envs.obs())
        if rew is not None:
            cmp(raw[:, O], rew)

    check(-1)
    resets = 0
    for t in range(Tn):
        zt = torch.as_tensor(z[t]).cuda().contiguous()
        call("mrl_rollout_act", d, int(_lib.HEAD_GAUSS), A, ptr(zt), ptr(logstd), ctypes.byref(bufs), t, stream())
        act = noise[t].astype(np.float32) * np.float32(1.0) + z[t]
        rew, done = envs.step(act)
        ept = envs.ep_t.copy()
        last = done | (ept + 1 >= envs.max_steps) | (t == Tn - 1)
        envs.ep_t = ept + 1
        if t < Tn - 1 and last.any():
            envs.reset(np.nonzero(last)[0])
            resets += int(last.sum())
        check(t, rew)
    assert resets > 0  # the auto-reset path ran
    print("humanoid step twin: max rel diff %.3g, %d of %d words differ" % tuple(worst))
    assert worst[0] <= 1e-7


def test_layered_rollout_graph_replay_equals_eager():
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    _, _, pol = _layered_policy("gauss", 376, 17, [256, 256], seed=3)
    outs = []
    for g in (False, True):
        col = Collector(env, pol, 256, 8, 1000, seed=9, use_graph=g)
        for _ in range(3):
            b = col.collect()
        outs.append((b.obs.clone(), b.act.clone(), b.rew.clone(), col.filter_state.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_humanoid_trpo_update_matches_oracle():
    """One TrpoUpdater.update on a Humanoid-shaped batch through the layered GEMM path:
    accepted k, lm, shs, theta and surr/kl/ent within 1e-4 relative of the oracle."""
    from modular_rl_amd.collector import Batch
    from modular_rl_amd.trpo import TrpoUpdater
    rng = np.random.default_rng(5)
    spec, th, pol = _layered_policy("gauss", 376, 17, [512, 512, 512], seed=8)
    N = 3000
    ob = rng.standard_normal((N, 376)).astype(np.float32).astype(np.float64)
    oldprob = T.policy_prob(spec, th, ob).astype(np.float32).astype(np.float64)
    act = T.sample(spec, oldprob, rng.standard_normal((N, 17))).astype(np.float32).astype(np.float64)
    adv = T.standardize(rng.standard_normal(N) + 0.5 * ob[:, 0]).astype(np.float32).astype(np.float64)
    th_w, stats_w, diag_w = T.trpo_update(spec, th, ob, act, adv, oldprob, cg_damping=0.1, max_kl=0.01)
    up = TrpoUpdater(pol, dict(cg_damping=0.1, max_kl=0.01))
    b = Batch(N, _dev(ob), _dev(act), _dev(oldprob))
    b.adv = _dev(adv)
    stats = up.update(b)
    dg = up.last_diag
    assert dg["k"] == diag_w["k"]
    np.testing.assert_allclose(dg["lm"], diag_w["lm"], rtol=1e-4)
    np.testing.assert_allclose(dg["shs"], diag_w["shs"], rtol=1e-4)
    th1 = pol.get_flat().astype(np.float64)
    assert np.abs(th1 - th_w).max() <= 1e-4 * np.abs(th_w - th).max() + 1e-7
    for k in ("surr_before", "surr_after", "kl_after", "ent_before", "ent_after"):
        np.testing.assert_allclose(stats[k], stats_w[k], rtol=1e-4, atol=1e-7, err_msg=k)


def test_humanoid_agent_iterations():
    """TrpoAgent on Humanoid-v2 with hid_sizes 512x3 (C5 net, reduced E/T): two full
    iterations (rollout, GAE, VF fit, TRPO step) run and stay within the trust region."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.core import run_policy_gradient_algorithm
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    cfg = dict(hid_sizes=[512, 512, 512], n_envs=128, horizon=64, timestep_limit=1000, n_iter=2, gamma=0.995,
               lam=0.97, max_kl=0.01, cg_damping=0.1, timesteps_per_batch=128 * 64, use_graph=1)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    assert agent.policy.net.layered and agent.baseline.reg.net.layered
    seen = []
    run_policy_gradient_algorithm(env, agent, callback=lambda st: seen.append(dict(st)), usercfg=cfg)
    assert len(seen) == 2
    for st in seen:
        assert np.isfinite(st["EpRewMean"]) and st["pol_kl_after"] <= 1.5 * 0.01


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_c5_width_rollout_invariants_and_update(dtype):
    """C5 at its per-GPU width (1024 Humanoid-v2 envs x 1024 steps, the
    376-512-512-512-17 policy, the wave-per-env step on all 256 CUs, captured graph):
    the size-independent properties of the lock-step batch (as the C3 full-size test:
    episode counters, terminations, the ZFilter clip and count, episode lengths adding up
    to the horizon, finite rewards, std = exp(logstd) rows), then one TRPO iteration whose
    step stays in the trust region: line search accepted, lm finite and positive, KL after
    the step within 2 max_kl, the surrogate improved."""
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.core import IterationRunner
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    E, Tn, max_kl = 1024, 1024, 0.01
    cfg = dict(timestep_limit=env.spec.max_episode_steps, gamma=0.995, lam=0.97, max_kl=max_kl, cg_damping=0.1,
               n_envs=E, horizon=Tn, filter=1, seed=3, hid_sizes=[512, 512, 512], activation="tanh", use_graph=1,
               mlp_dtype=dtype)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    col = agent.make_collector(env, cfg)
    assert col.layered and col.wave_per_env
    runner = IterationRunner(agent, col, cfg, pipeline=False)
    stats = runner.step()
    torch.cuda.synchronize()
    flags = col.flags.cpu().numpy().reshape(Tn, E)
    ep_t = col.ep_t.cpu().numpy().reshape(Tn, E).astype(np.int64)
    last, term = (flags & 1) > 0, (flags & 2) > 0
    assert not (term & ~last).any()
    assert (ep_t[0] == 0).all() and last[-1].all()
    np.testing.assert_array_equal(ep_t[1:], np.where(last[:-1], 0, ep_t[:-1] + 1))
    np.testing.assert_array_equal(np.where(last, ep_t + 1, 0).sum(0), np.full(E, Tn))
    assert term.any()  # the articulated Humanoid falls within the horizon under a random policy
    obs = col.obs.cpu().numpy()
    assert np.isfinite(obs).all() and np.abs(obs).max() <= 5.0
    (n, _, var), (nr, _, _) = col.filter_stats()
    assert n == E * Tn and nr == E * Tn and np.isfinite(var).all()
    assert np.isfinite(col.rew.cpu().numpy()).all()
    prob = col.prob.cpu().numpy().reshape(Tn * E, -1)
    np.testing.assert_array_equal(prob[:, 17:], np.broadcast_to(prob[:1, 17:], prob[:, 17:].shape))
    # the update
    dg = agent.updater.last_diag
    assert dg["success"] and 0 <= dg["k"] < 10, dg
    assert np.isfinite(dg["lm"]) and dg["lm"] > 0
    assert 0 <= stats["pol_kl_after"] <= 2 * max_kl, stats["pol_kl_after"]
    assert stats["pol_surr_after"] < stats["pol_surr_before"]
    assert np.isfinite(stats["vf_loss_after"]) and stats["vf_loss_after"] <= stats["vf_loss_before"]


@pytest.mark.parametrize("E,Tn,hid", [(1026, 6, [256, 256]), (64, 60, [64, 64])])
def test_humanoid_four_envs_per_block_equals_one(E, Tn, hid, monkeypatch):
    """MRL_HM_WPB=4 (four env waves per Humanoid block, the wave state in dynamic LDS, the
    model tables loaded once per block; the default) against one-wave blocks: the same
    per-env arithmetic, so flags, observations, actions, rewards and the filter state
    agree bit for bit -- a ragged last block (1026 = 256 x 4 + 2) and mid-horizon
    terminations with auto-reset (64 envs x 60 steps)."""
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    _, _, pol = _layered_policy("gauss", 376, 17, hid, seed=5)
    outs = []
    for wpb in ("1", "4"):
        monkeypatch.setenv("MRL_HM_WPB", wpb)
        col = Collector(env, pol, E, Tn, 1000, seed=11, use_graph=False)
        for _ in range(2):
            b = col.collect()
        torch.cuda.synchronize()
        outs.append((b.flags.clone(), b.obs.clone(), b.act.clone(), b.rew.clone(), col.filter_state.clone()))
    if Tn >= 60:
        assert ((outs[0][0] & 2) != 0).any()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
