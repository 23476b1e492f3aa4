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
