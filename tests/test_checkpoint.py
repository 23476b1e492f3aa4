"""Checkpoint / resume and run-log format.  CPU tests use a stand-in
agent with host tensors (format and restore logic); the GPU test checks that a run
resumed from a snapshot continues bit-identically to the uninterrupted run."""
import json

import numpy as np
import pytest
import torch

from modular_rl_amd.checkpoint import RunLog, apply_collector_state, load_snapshot, save_snapshot


class _Net:
    def __init__(self, P, seed):
        self.P = P
        self.theta = torch.as_tensor(np.random.default_rng(seed).standard_normal(P), dtype=torch.float32)

    def set_flat(self, th):
        self.theta.copy_(torch.as_tensor(np.asarray(th), dtype=torch.float32))


class _Col:
    def __init__(self, E, FS, seed):
        rng = np.random.default_rng(seed)
        self.E, self.FS = E, FS
        self.filter_state = torch.as_tensor(rng.standard_normal(2 * FS))
        self.iteration = torch.tensor([int(rng.integers(0, 100))], dtype=torch.int64)
        self.env_int = torch.as_tensor(rng.integers(0, 50, size=2 * E), dtype=torch.int32)


class _Agent:
    def __init__(self, seed, with_col=True):
        self.policy = type("P", (), {"net": _Net(37, seed)})()
        self.baseline = type("B", (), {"net": _Net(29, seed + 1)})()
        self.cfg = {"gamma": 0.995, "hid_sizes": [64, 64], "obj": object()}
        self._col = _Col(8, 14, seed + 2) if with_col else None
        self._pending_state = None

    def _filter_owner(self):
        return self._col


def test_snapshot_roundtrip_restores_params_filter_and_rng(tmp_path):
    a, b = _Agent(1), _Agent(2)
    path = save_snapshot(str(tmp_path / "s.npz"), a, counter=7, env_id="Hopper-v2")
    meta = load_snapshot(path, b)
    assert meta["counter"] == 7 and meta["env_id"] == "Hopper-v2" and meta["cfg"]["gamma"] == 0.995
    assert torch.equal(a.policy.net.theta, b.policy.net.theta)
    assert torch.equal(a.baseline.net.theta, b.baseline.net.theta)
    assert torch.equal(a._col.filter_state[:a._col.FS], b._col.filter_state[:b._col.FS])
    assert torch.equal(a._col.iteration, b._col.iteration)
    assert torch.equal(a._col.env_int[8:], b._col.env_int[8:])
    # the file holds plain arrays only
    with np.load(path, allow_pickle=False) as z:
        assert set(z.files) >= {"policy__theta", "vf__theta", "filter__state", "rng__iteration", "meta"}


def test_snapshot_state_waits_for_the_first_collector(tmp_path):
    a, b = _Agent(3), _Agent(4, with_col=False)
    path = save_snapshot(str(tmp_path / "s.npz"), a, counter=2)
    load_snapshot(path, b)
    assert b._pending_state is not None and "filter/state" in b._pending_state
    col = _Col(8, 14, 9)
    apply_collector_state(col, b._pending_state)
    assert torch.equal(col.filter_state[:14], a._col.filter_state[:14])


def test_snapshot_rejects_mismatched_nets(tmp_path):
    a = _Agent(5)
    path = save_snapshot(str(tmp_path / "s.npz"), a)
    b = _Agent(6)
    b.policy.net = _Net(40, 0)
    with pytest.raises(ValueError):
        load_snapshot(path, b)


def test_run_log_npz_layout(tmp_path):
    log = RunLog(str(tmp_path / "run.h5"), {"seed": 0, "env": "Hopper-v2"})
    log.h5 = False
    for i in range(3):
        log.record({"EpRewMean": float(i), "pol_kl_after": 0.01 * i})
    log.snapshot(3, _Agent(7), "Hopper-v2")
    out = log.save()
    with np.load(out, allow_pickle=False) as z:
        np.testing.assert_array_equal(z["diagnostics__EpRewMean"], [0.0, 1.0, 2.0])
        assert json.loads(bytes(z["params"]).decode())["env"] == "Hopper-v2"
        assert "agent_snapshots__0003__policy__theta" in z.files


@pytest.mark.gpu
@pytest.mark.parametrize("agent_name,pipeline", [("TrpoAgent", 1), ("TrpoAgent", 0), ("PpoLbfgsAgent", 1),
                                                 ("PpoSgdAgent", 1)])
def test_resume_continues_bit_identically(tmp_path, agent_name, pipeline):
    """A snapshot taken INSIDE the iteration-2 callback (as run_pg.py takes them) and
    resumed for one iteration ends bit-identical to the uninterrupted 3-iteration run:
    parameters, VF, the updater's state (PPO kl_coeff / Adam moments) and the stats.
    With pipeline=1 the callback fires after iteration 3 is already issued, so this
    checks the runner's end-of-iteration capture."""
    from modular_rl_amd import agentzoo
    from modular_rl_amd.core import run_policy_gradient_algorithm
    from modular_rl_amd.envs import make
    env = make("Hopper-v2")
    cfg = dict(n_envs=64, horizon=64, timestep_limit=1000, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1,
               timesteps_per_batch=64 * 64, use_graph=1, seed=3, pipeline=pipeline, epochs=2, kl_target=0.003)
    Agent = getattr(agentzoo, agent_name)
    path = str(tmp_path / "snap.npz")

    def run(agent, n, snap_at=None):
        seen = []

        def cb(st):
            seen.append(dict(st))
            if len(seen) == snap_at:
                save_snapshot(path, agent, counter=snap_at, env_id="Hopper-v2")
        run_policy_gradient_algorithm(env, agent, callback=cb, usercfg=dict(cfg, n_iter=n))
        return seen

    full = Agent(env.observation_space, env.action_space, cfg)
    st_full = run(full, 3, snap_at=2)
    resumed = Agent(env.observation_space, env.action_space, cfg)
    meta = load_snapshot(path, resumed)
    assert meta["counter"] == 2
    st_res = run(resumed, 1)
    assert np.array_equal(resumed.policy.get_flat(), full.policy.get_flat())
    assert np.array_equal(resumed.baseline.net.get_flat(), full.baseline.net.get_flat())
    if hasattr(full.updater, "state_arrays"):
        for k, v in full.updater.state_arrays().items():
            w = resumed.updater.state_arrays()[k]
            a = v.cpu().numpy() if torch.is_tensor(v) else v
            b = w.cpu().numpy() if torch.is_tensor(w) else w
            assert np.array_equal(a, b), k
    for k in ("EpRewMean", "pol_surr_after", "pol_kl_after", "vf_EVBefore"):
        if k in st_full[-1]:
            assert st_res[0][k] == st_full[-1][k], k


def test_updater_state_roundtrip(tmp_path):
    """PPO updater state (kl_coeff, Adam m / v / t) is saved and restored as arrays."""
    class _Upd:
        def __init__(self, seed):
            rng = np.random.default_rng(seed)
            self.kl_coeff = float(rng.random())
            self.m = torch.as_tensor(rng.standard_normal(37), dtype=torch.float32)
            self.t = int(rng.integers(1, 100))

        def state_arrays(self):
            return {"kl_coeff": np.array([self.kl_coeff]), "adam_m": self.m, "adam_t": np.array([self.t])}

        def load_state_arrays(self, st):
            self.kl_coeff = float(st["kl_coeff"][0])
            self.m.copy_(torch.as_tensor(st["adam_m"]))
            self.t = int(st["adam_t"][0])

    a, b = _Agent(11), _Agent(12)
    a.updater, b.updater = _Upd(1), _Upd(2)
    load_snapshot(save_snapshot(str(tmp_path / "u.npz"), a), b)
    assert b.updater.kl_coeff == a.updater.kl_coeff and b.updater.t == a.updater.t
    assert torch.equal(b.updater.m, a.updater.m)


def test_episode_counters_of_another_env_count_are_refused(tmp_path):
    a = _Agent(13)
    path = save_snapshot(str(tmp_path / "e.npz"), a)
    b = _Agent(14, with_col=False)
    load_snapshot(path, b)
    with pytest.raises(ValueError):
        apply_collector_state(_Col(16, 14, 0), b._pending_state)


def test_capture_in_two_parts_equals_one():
    """The runner captures the state the next rollout advances before issuing it
    (capture_state(host=False)) and the host-only rest after (capture_host_state): the
    two parts hold exactly the keys and values of one whole capture."""
    from modular_rl_amd.checkpoint import capture_host_state, capture_state
    a = _Agent(5)
    whole = capture_state(a)
    dev = capture_state(a, host=False)
    host = capture_host_state(a)
    assert not set(dev) & set(host) and set(dev) | set(host) == set(whole)
    assert all(k.startswith(("policy/", "vf/", "filter/", "rng/iteration", "rng/episodes")) for k in dev)
    for k, v in {**dev, **host}.items():
        w = whole[k]
        assert (torch.equal(v, w) if torch.is_tensor(v) else np.array_equal(v, w)), k
