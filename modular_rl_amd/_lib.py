"""ctypes binding of libmrl_hip.so (the C ABI declared in include/mrl_hip.h).

There is no CPU fallback: if the library is missing or no GPU is visible the
product path raises ``MrlError`` (the oracle in ``oracle/`` is test-only).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# MRL_LIB_PATH: diagnostic override (ablation builds under tools/); the default is the in-tree build
_DEFAULT_PATH = os.path.join(_HERE, "libmrl_hip.so")
LIB_PATH = os.environ.get("MRL_LIB_PATH") or _DEFAULT_PATH

OK = 0
HEAD_LINEAR, HEAD_SOFTMAX, HEAD_GAUSS = 0, 1, 2
CACHE_NONE, CACHE_WRITE, CACHE_READ = 0, 1, 2
EPI_PROB, EPI_LOSSES, EPI_SURRGRAD, EPI_VFLOSS, EPI_FVP, EPI_PPOGRAD, EPI_PPOSGD = 0, 1, 2, 3, 4, 5, 6
PPO_BLOCK_ROWS = 128
ENV_CARTPOLE, ENV_HOPPER, ENV_HUMANOID = 0, 1, 2
GEMM_STORE, GEMM_TANH, GEMM_DTANH, GEMM_SLAB = 0, 1, 2, 3
COMPUTE_F32, COMPUTE_BF16, COMPUTE_SPLIT = 0, 1, 2
COMPUTE = {"fp32": COMPUTE_F32, "bf16": COMPUTE_BF16}

vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f64 = ctypes.c_double


class MrlError(RuntimeError):
    pass


class MlpDesc(ctypes.Structure):
    _fields_ = [("n_in", i32), ("n_out", i32), ("head", i32), ("n_hidden", i32), ("n_layers", i32), ("cus", i32)]


class RowsIO(ctypes.Structure):
    _fields_ = [("x", vp), ("ep_t", vp), ("timestep_limit", f64), ("n", i64), ("inv_n_global", f64),
                ("act", vp), ("adv", vp), ("oldprob", vp), ("target", vp), ("out", vp), ("ghead", vp),
                ("partial", vp), ("kl_coeff", f64), ("kl_cutoff", f64), ("cutoff_coeff", f64), ("reverse_kl", i32),
                ("cache_mode", i32), ("act_cache", vp), ("feat_out", vp)]


class GemmDesc(ctypes.Structure):
    _fields_ = [("m", i64), ("n", i64), ("k", i64), ("a", vp), ("lda", i64), ("a_trans", i32), ("ones_row", i32),
                ("b", vp), ("ldb", i64), ("b_trans", i32), ("epilogue", i32), ("a2", vp), ("b2", vp), ("c", vp),
                ("ldc", i64), ("bias", vp), ("h", vp), ("ldh", i64), ("splits", i32), ("compute", i32),
                ("slab_stride", i64)]


class GemmBf16Desc(ctypes.Structure):
    _fields_ = [("m", i64), ("n", i64), ("k", i64), ("a", vp), ("lda", i64), ("bt", vp), ("ldb", i64), ("a2", vp),
                ("bt2", vp), ("c", vp), ("ldc", i64), ("c_bf16", i32), ("epilogue", i32), ("bias", vp), ("h", vp),
                ("ldh", i64), ("lds_limit", i32)]


class GemmBf16TnDesc(ctypes.Structure):
    _fields_ = [("m", i64), ("n", i64), ("k", i64), ("a", vp), ("lda", i64), ("b", vp), ("ldb", i64),
                ("ones_row", i32), ("splits", i32), ("slab", vp), ("slab_stride", i64), ("ldc", i64),
                ("lds_limit", i32)]


class RolloutDesc(ctypes.Structure):
    _fields_ = [("env_id", i32), ("n_envs", i32), ("horizon", i32), ("timestep_limit", i32), ("filter", i32),
                ("env_offset", i32), ("seed", ctypes.c_uint64), ("compute", i32), ("launch_cus", i32)]


class RolloutBufs(ctypes.Structure):
    _fields_ = [("env_state", vp), ("env_int", vp), ("filter_state", vp), ("records", vp), ("iteration", vp),
                ("obs", vp), ("act", vp), ("prob", vp), ("rew", vp), ("flags", vp), ("ep_t", vp), ("noise", vp),
                ("stamps", vp), ("raw_obs", vp), ("obs_bf16", vp)]


# name -> (restype, argtypes); every symbol include/mrl_hip.h declares
SIGNATURES = {
    "mrl_last_error": (ctypes.c_char_p, []),
    "mrl_version": (i32, []),
    "mrl_mlp_num_params": (i64, [vp]),
    "mrl_mlp_image_floats": (i64, [vp]),
    "mrl_mlp_pack": (i32, [vp, vp, vp, i32, vp, vp]),
    "mrl_partial_rows": (i64, [i64]),
    "mrl_act_cache_floats": (i64, [i64]),
    "mrl_slab_rows": (i64, [i64]),
    "mrl_mlp_partial_rows": (i64, [vp, i64]),
    "mrl_mlp_slab_rows": (i64, [vp, i64]),
    "mrl_mlp_rows": (i32, [vp, i32, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_mlp_vjp": (i32, [vp, vp, vp, vp, f64, vp, i64, vp, vp, vp, vp]),
    "mrl_mlp_image_words_bf16": (i64, [vp]),
    "mrl_act_cache_words_bf16": (i64, [i64]),
    "mrl_partial_rows_bf16": (i64, [i64]),
    "mrl_slab_rows_bf16": (i64, [i64]),
    "mrl_mlp_partial_rows_bf16": (i64, [vp, i64]),
    "mrl_mlp_slab_rows_bf16": (i64, [vp, i64]),
    "mrl_mlp_pack_bf16": (i32, [vp, vp, vp, i32, vp, vp]),
    "mrl_mlp_rows_bf16": (i32, [vp, i32, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_mlp_vjp_bf16": (i32, [vp, vp, vp, vp, f64, vp, i64, vp, vp, vp, vp]),
    "mrl_mlp_image_words_split": (i64, [vp]),
    "mrl_mlp_pack_split": (i32, [vp, vp, vp, vp, vp]),
    "mrl_mlp_fisher_hyb_fits": (i32, [vp]),
    "mrl_mlp_rows_split": (i32, [vp, i32, vp, vp, vp, vp, vp]),
    "mrl_mlp_fisher_hyb": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_mlp_grad_hyb": (i32, [vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_mlp_fvp_split": (i32, [vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_reduce_rows_f32": (i32, [vp, i64, i64, vp, vp, vp]),
    "mrl_reduce_rows_f64": (i32, [vp, i64, i64, vp, vp, vp]),
    "mrl_gemm": (i32, [vp, vp, vp]),
    "mrl_gemm_slab_splits": (i64, [i64, i32]),
    "mrl_gemm_tile_n": (i32, [vp]),
    "mrl_gemm_bf16": (i32, [vp, vp, vp]),
    "mrl_gemm_bf16_tn": (i32, [vp, vp, vp]),
    "mrl_cast_rows_bf16": (i32, [vp, i64, i64, i64, vp, i64, vp]),
    "mrl_pack_w_bf16": (i32, [vp, i64, i64, i32, vp, i64, vp]),
    "mrl_colsum": (i32, [vp, i64, i64, i64, i32, vp, i64, vp, vp]),
    "mrl_head_rows": (i32, [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_concat_time": (i32, [vp, vp, i64, i32, f64, vp, i32, vp]),
    "mrl_cg_state_doubles": (i64, [i64]),
    "mrl_cg_init": (i32, [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_cg_update": (i32, [vp, f64, f64, i64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_cg_update_pack": (i32, [vp, f64, f64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_trpo_step": (i32, [vp, vp, vp, f64, f64, i64, vp, vp, vp]),
    "mrl_trpo_step_ax": (i32, [vp, vp, vp, f64, i64, vp, vp, vp]),
    "mrl_device_cu_count": (i32, [vp]),
    "mrl_stream_create_cu_mask": (i32, [vp, i32, vp]),
    "mrl_stream_get_cu_mask": (i32, [vp, i32, vp]),
    "mrl_stream_destroy": (i32, [vp]),
    "mrl_stream_signal": (i32, [vp, vp, ctypes.c_uint32]),
    "mrl_stream_wait": (i32, [vp, vp, ctypes.c_uint32]),
    "mrl_axpy_cast": (i32, [vp, vp, f64, i64, vp, vp]),
    "mrl_linesearch_candidates": (i32, [vp, vp, i32, i32, i64, vp, vp]),
    "mrl_linesearch_eval": (i32, [vp, i32, vp, vp, i32, i32, vp, vp, vp, i64, vp, i64, vp, vp]),
    "mrl_cast_scale_f32_f64": (i32, [vp, f64, i64, vp, vp]),
    "mrl_adam_step": (i32, [vp, vp, vp, vp, f64, f64, f64, f64, i64, vp]),
    "mrl_gather_rows": (i32, [vp, vp, i64, i64, vp, vp]),
    "mrl_gae": (i32, [vp, vp, vp, i64, i64, f64, f64, vp, vp, vp, vp, vp]),
    "mrl_gae_workspace_bytes": (i64, [i64, i64]),
    "mrl_standardize": (i32, [vp, i64, vp, vp, vp]),
    "mrl_vf_target": (i32, [vp, vp, f64, i64, vp, vp]),
    "mrl_moments": (i32, [vp, vp, i64, vp, vp, vp]),
    "mrl_moments_centered": (i32, [vp, vp, i64, vp, vp, vp, vp]),
    "mrl_probtype_rows": (i32, [i32, i32, i64, vp, vp, vp, vp, vp, vp, vp]),
    "mrl_moments_workspace_bytes": (i64, [i64]),
    "mrl_episode_stats": (i32, [vp, vp, i64, i64, vp, vp, vp]),
    "mrl_episode_stats_workspace_bytes": (i64, [i64]),
    "mrl_env_state_doubles": (i64, [i32]),
    "mrl_filter_doubles": (i64, [i32]),
    "mrl_record_doubles": (i64, [i32]),
    "mrl_rollout_blocks": (i64, [i32]),
    "mrl_rollout_reset": (i32, [vp, vp, vp]),
    "mrl_rollout_noise_doubles": (i64, [vp]),
    "mrl_rollout_noise": (i32, [vp, vp, vp, vp]),
    "mrl_rollout_image_floats": (i64, [vp]),
    "mrl_rollout_pack": (i32, [vp, vp, vp, vp, vp]),
    "mrl_rollout_step": (i32, [vp, vp, vp, vp, vp, i32, vp]),
    "mrl_rollout_sync_bytes": (i64, [vp]),
    "mrl_rollout_run": (i32, [vp, vp, vp, vp, vp, vp, i32, vp]),
    "mrl_rollout_finish": (i32, [vp, vp, vp]),
    "mrl_rollout_reset_rows": (i32, [vp, vp, vp]),
    "mrl_rollout_obs": (i32, [vp, vp, i32, vp]),
    "mrl_rollout_act": (i32, [vp, i32, i32, vp, vp, vp, i32, vp]),
    "mrl_rollout_act_head": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp]),
    "mrl_rollout_act_head_bf16": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp]),
}

_lib = None


def load(require_gpu=False):
    """Load libmrl_hip.so once; raise MrlError if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MrlError(f"{LIB_PATH} is not built: run `make` (or __graft_entry__.build()); "
                           "modular_rl_amd has no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if LIB_PATH != _DEFAULT_PATH and not hasattr(lib, name):
                continue  # an ablation build that predates this entry point
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_gpu and not torch.cuda.is_available():
        raise MrlError("modular_rl_amd needs a ROCm GPU (MI355X); none is visible and there is no CPU fallback")
    return _lib


def check(rc, what=""):
    if rc != OK:
        msg = load().mrl_last_error().decode()
        raise MrlError(f"{what}: rc={rc}: {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def call(name, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
