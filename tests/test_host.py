"""Host-side plumbing that mirrors the reference API (no GPU needed)."""
import argparse

import numpy as np

from modular_rl_amd import misc_utils as MU


def test_option_tuples_and_defaults_match_reference():
    from modular_rl_amd.agentzoo import FILTER_OPTIONS, MLP_OPTIONS, TrpoAgent
    from modular_rl_amd.core import PG_OPTIONS
    from modular_rl_amd.trpo import TrpoUpdater
    names = [o[0] for o in TrpoAgent.options]
    # reference: MLP_OPTIONS + PG_OPTIONS + TrpoUpdater.options + FILTER_OPTIONS (agentzoo.py:126)
    for ref in ["hid_sizes", "activation", "timestep_limit", "n_iter", "parallel", "timesteps_per_batch", "gamma",
                "lam", "cg_damping", "max_kl", "filter"]:
        assert ref in names
    d = MU.update_default_config(TrpoAgent.options, {"gamma": 0.995, "unknown": 1})
    assert d.gamma == 0.995 and d.lam == 1.0 and d.cg_damping == 1e-3 and d.max_kl == 1e-2
    assert d.timesteps_per_batch == 100 and d.hid_sizes == [64, 64] and d.filter == 1
    assert "unknown" not in d
    assert [o[0] for o in TrpoUpdater.options] == ["cg_damping", "max_kl"]
    assert MLP_OPTIONS[0][0] == "hid_sizes" and FILTER_OPTIONS[0][0] == "filter"
    assert [o[0] for o in PG_OPTIONS][:6] == ["timestep_limit", "n_iter", "parallel", "timesteps_per_batch", "gamma",
                                              "lam"]


def test_argument_parser_two_phase():
    from modular_rl_amd.agentzoo import TrpoAgent
    p = argparse.ArgumentParser()
    MU.update_argument_parser(p, MU.GENERAL_OPTIONS)
    MU.update_argument_parser(p, TrpoAgent.options)
    a = p.parse_args(["--hid_sizes", "64,64", "--max_kl", "0.02", "--n_envs", "8"])
    assert a.hid_sizes == [64, 64] and a.max_kl == 0.02 and a.n_envs == 8 and a.seed == 0


def test_comma_sep_ints_is_a_list():
    assert MU.comma_sep_ints("10,5") == [10, 5]
    assert MU.comma_sep_ints("") == []


def test_get_agent_cls_and_env_registry():
    from modular_rl_amd.core import get_agent_cls, horizon_of
    from modular_rl_amd.envs import Box, Discrete, make
    assert get_agent_cls("modular_rl_amd.agentzoo.TrpoAgent").__name__ == "TrpoAgent"
    e = make("Hopper-v2")
    assert isinstance(e.observation_space, Box) and e.observation_space.shape == (11,)
    assert isinstance(e.action_space, Box) and e.action_space.shape == (3,) and e.spec.max_episode_steps == 1000
    c = make("CartPole-v0")
    assert isinstance(c.action_space, Discrete) and c.action_space.n == 2 and c.spec.max_episode_steps == 200
    assert horizon_of({"timesteps_per_batch": 100, "n_envs": 8, "horizon": 0}) == 13
    assert horizon_of({"timesteps_per_batch": 100, "n_envs": 8, "horizon": 32}) == 32


def test_paths_batch_roundtrip_flags():
    """Per-path dicts -> time-major flags (bit0 last, bit1 terminated) as the GAE kernel expects."""
    from modular_rl_amd.collector import Batch
    paths = [dict(observation=np.zeros((3, 2)), reward=np.ones(3), terminated=True),
             dict(observation=np.zeros((2, 2)), reward=np.ones(2), terminated=False)]
    b = Batch.from_paths(paths, None, device="cpu", need_policy=False)
    assert b.flags.tolist() == [0, 0, 3, 0, 1]
    assert b.ep_t.tolist() == [0, 1, 2, 0, 1]
    assert b.T == 5 and b.E == 1


def test_mlp_dtype_option_and_validation():
    """mlp_dtype (the bf16 throughput mode) is an MLP option defaulting to fp32, the
    parity dtype; an unknown dtype is rejected before any device work."""
    import pytest

    from modular_rl_amd import _lib
    from modular_rl_amd.agentzoo import MLP_OPTIONS, TrpoAgent
    from modular_rl_amd.nets import check_dtype
    assert ("mlp_dtype" in [o[0] for o in MLP_OPTIONS])
    d = MU.update_default_config(TrpoAgent.options, {})
    assert d.mlp_dtype == "fp32"
    assert check_dtype("bf16") == "bf16" and check_dtype("fp32") == "fp32"
    with pytest.raises(_lib.MrlError):
        check_dtype("fp16")
    assert _lib.COMPUTE == {"fp32": _lib.COMPUTE_F32, "bf16": _lib.COMPUTE_BF16}


def test_bench_flop_and_byte_accounting():
    """bench.py's algorithmic work per row of the Fisher-product kernels (the roofline
    numerators): fused 11-64-64-3 net, JVP and VJP 18,560 FLOP each with the cache."""
    import types

    import bench
    net = types.SimpleNamespace(n_in=11, n_out=3, hid_sizes=[64, 64], layered=False, use_cache=True)
    f = bench.flops_per_row(net)
    assert f["fvp_jvp_rows"] == 18560 and f["fvp_vjp"] == 18560 and f["policy_forward"] == 2 * (11 * 64 + 64 * 64 + 64 * 3)
    hum = types.SimpleNamespace(n_in=376, n_out=17, hid_sizes=[512, 512, 512], layered=True)
    assert bench.flops_per_row(hum)["fvp_vjp"] == 2516992


def test_bench_roofline_kernel_is_chosen_per_binary():
    """The VJP binary's roles are summed like rocprofv3 sums one kernel name, and the
    roofline kernel is the binary with the largest device time per iteration."""
    import bench
    rows, K = 1000, 2
    kern = {"fvp_vjp": (20, 1.0, 20.0), "pg_vjp": (2, 1.0, 2.0), "vf_vjp": (6, 1.5, 9.0)}
    e = bench.vjp_binary_entry(kern, 100.0, 80.0, rows, K)
    assert e["launches"] == 28 and e["total_ms"] == 31.0 and abs(e["mean_ms"] - 31.0 / 28) < 1e-12
    assert abs(e["flop_per_row"] - (22 * 100.0 + 6 * 80.0) / 28) < 1e-9
    assert e["roles"]["vf_vjp"] == {"launches": 6, "mean_ms": 1.5, "ms_per_iter": 4.5}
    assert bench.vjp_binary_entry({"pg_vjp": (2, 1.0, 2.0)}, 100.0, 80.0, rows, K) is None
    assert bench.vjp_binary_entry(kern, 100.0, None, rows, K)["launches"] == 22  # layered VF: not this binary
    kinfo = {"fvp_vjp": {"total_ms": 20.0}, "mlp_vjp16_kernel": {"total_ms": 31.0}, "rollout_step": {"total_ms": 27.0},
             "fvp_jvp_rows": {"total_ms": 15.0}}
    assert bench.dominant_kernel(kinfo) == "mlp_vjp16_kernel"
    kinfo["rollout_step"]["total_ms"] = 40.0
    assert bench.dominant_kernel(kinfo) == "rollout_step"
    # without the binary entry (layered nets) the Fisher-product role competes itself
    assert bench.dominant_kernel({"fvp_vjp": {"total_ms": 50.0}, "rollout_step": {"total_ms": 40.0}}) == "fvp_vjp"


def test_rollout_cu_split(monkeypatch):
    """The pipelined loop's CU sets: the rollout's blocks first, the VF fit on the rest
    (or on MRL_FIT_CUS of them); no split when the rollout wants more than half."""
    from modular_rl_amd.core import rollout_cu_split
    r, f = rollout_cu_split(64, 256)
    assert r == list(range(64)) and f == list(range(64, 256))
    assert rollout_cu_split(200, 256) is None and rollout_cu_split(0, 256) is None
    monkeypatch.setenv("MRL_FIT_CUS", "96")
    r, f = rollout_cu_split(64, 256)
    assert r == list(range(64)) and f == list(range(64, 160))


def test_timing_samples_detail_regions_every_nth_iteration():
    """bench.py's timing: per-launch ("detail") regions and the phase events only on every
    detail_every-th iteration (each HIP timing event is a queue marker that delays the
    next kernel); the bookkeeping alone, no events recorded (no GPU here)."""
    from modular_rl_amd import timing
    timing.enable(True, detail_every=4)
    try:
        seen = []
        for _ in range(9):
            timing.tick()
            seen.append(timing.detail_now())
        assert seen == [True, False, False, False, True, False, False, False, True]
        assert timing._iters == 9 and timing._detail_iters == 3
        # an unsampled iteration records nothing for a detail region and drop_last leaves
        # the sampled iterations' records alone
        timing.tick()
        assert not timing.detail_now()
        timing._events["fvp_onepass"].append(("a", "b"))
        timing._detail_names.add("fvp_onepass")
        timing.drop_last("fvp_onepass", 1)
        assert len(timing._events["fvp_onepass"]) == 1
    finally:
        timing.enable(False)
    assert not timing.detail_now()
