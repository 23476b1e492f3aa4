"""The C-ABI boundary without a GPU: libmrl_hip.so loads, exports every function
include/mrl_hip.h declares, the ctypes binding matches the C struct layouts
(compiled probe with gcc), host-only queries answer, and the product path refuses
to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mrl_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mrl_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from modular_rl_amd import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 30
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mrl_[a-z0-9_]+)", nm))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    unbound = [n for n in names if n not in _lib.SIGNATURES]
    assert not unbound, unbound
    for n in names:
        assert getattr(lib, n) is not None


def test_ctypes_struct_layout_matches_c(tmp_path):
    from modular_rl_amd import _lib
    probe = tmp_path / "probe.c"
    probe.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "mrl_hip.h"
#define P(T, F) printf(#T "." #F " %zu\\n", offsetof(T, F));
int main(void) {
  printf("mrl_mlp_desc %zu\\nmrl_rows_io %zu\\nmrl_rollout_desc %zu\\nmrl_rollout_bufs %zu\\nmrl_gemm_desc %zu\\n",
         sizeof(mrl_mlp_desc), sizeof(mrl_rows_io), sizeof(mrl_rollout_desc), sizeof(mrl_rollout_bufs),
         sizeof(mrl_gemm_desc));
  P(mrl_gemm_desc, ones_row) P(mrl_gemm_desc, epilogue) P(mrl_gemm_desc, ldh) P(mrl_gemm_desc, slab_stride)
  P(mrl_rows_io, timestep_limit) P(mrl_rows_io, n) P(mrl_rows_io, inv_n_global) P(mrl_rows_io, partial)
  P(mrl_rows_io, act_cache) P(mrl_rows_io, feat_out)
  P(mrl_rollout_desc, seed) P(mrl_rollout_bufs, noise)
  printf("mrl_gemm_bf16_desc %zu\\nmrl_gemm_bf16_tn_desc %zu\\n", sizeof(mrl_gemm_bf16_desc),
         sizeof(mrl_gemm_bf16_tn_desc));
  P(mrl_gemm_bf16_desc, c_bf16) P(mrl_gemm_bf16_desc, bias) P(mrl_gemm_bf16_desc, ldh)
  P(mrl_gemm_bf16_tn_desc, ones_row) P(mrl_gemm_bf16_tn_desc, slab) P(mrl_gemm_bf16_tn_desc, ldc)
  return 0;
}
""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(probe), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n") if l)
    assert int(out["mrl_mlp_desc"]) == ctypes.sizeof(_lib.MlpDesc)
    assert int(out["mrl_rows_io"]) == ctypes.sizeof(_lib.RowsIO)
    assert int(out["mrl_rollout_desc"]) == ctypes.sizeof(_lib.RolloutDesc)
    assert int(out["mrl_rollout_bufs"]) == ctypes.sizeof(_lib.RolloutBufs)
    assert int(out["mrl_rows_io.timestep_limit"]) == _lib.RowsIO.timestep_limit.offset
    assert int(out["mrl_rows_io.n"]) == _lib.RowsIO.n.offset
    assert int(out["mrl_rows_io.inv_n_global"]) == _lib.RowsIO.inv_n_global.offset
    assert int(out["mrl_rows_io.partial"]) == _lib.RowsIO.partial.offset
    assert int(out["mrl_rows_io.act_cache"]) == _lib.RowsIO.act_cache.offset
    assert int(out["mrl_rows_io.feat_out"]) == _lib.RowsIO.feat_out.offset
    assert int(out["mrl_rollout_desc.seed"]) == _lib.RolloutDesc.seed.offset
    assert int(out["mrl_rollout_bufs.noise"]) == _lib.RolloutBufs.noise.offset
    assert int(out["mrl_gemm_desc"]) == ctypes.sizeof(_lib.GemmDesc)
    for f in ("ones_row", "epilogue", "ldh", "slab_stride"):
        assert int(out["mrl_gemm_desc." + f]) == getattr(_lib.GemmDesc, f).offset, f
    assert int(out["mrl_gemm_bf16_desc"]) == ctypes.sizeof(_lib.GemmBf16Desc)
    assert int(out["mrl_gemm_bf16_tn_desc"]) == ctypes.sizeof(_lib.GemmBf16TnDesc)
    for f in ("c_bf16", "bias", "ldh"):
        assert int(out["mrl_gemm_bf16_desc." + f]) == getattr(_lib.GemmBf16Desc, f).offset, f
    for f in ("ones_row", "slab", "ldc"):
        assert int(out["mrl_gemm_bf16_tn_desc." + f]) == getattr(_lib.GemmBf16TnDesc, f).offset, f


def test_host_queries_match_the_reference_parameter_layout():
    from modular_rl_amd import _lib
    from oracle import trpo_np as T
    lib = _lib.load()
    for (n_in, n_out, head, name) in [(11, 3, _lib.HEAD_GAUSS, "gauss"), (4, 2, _lib.HEAD_SOFTMAX, "softmax"),
                                      (12, 1, _lib.HEAD_LINEAR, "linear")]:
        d = _lib.MlpDesc(n_in, n_out, head, 64, 2)
        assert lib.mrl_mlp_num_params(ctypes.byref(d)) == T.Spec(n_in, [64, 64], n_out, name).P
        assert lib.mrl_mlp_image_floats(ctypes.byref(d)) > 0
    # Hopper 5,126 / CartPole 4,610 / VF 5,057 params
    assert lib.mrl_mlp_num_params(ctypes.byref(_lib.MlpDesc(11, 3, _lib.HEAD_GAUSS, 64, 2))) == 5126
    bad = _lib.MlpDesc(11, 3, _lib.HEAD_GAUSS, 128, 2)
    assert lib.mrl_mlp_num_params(ctypes.byref(bad)) < 0
    assert b"hid_sizes" in lib.mrl_last_error()
    assert lib.mrl_env_state_doubles(_lib.ENV_HOPPER) == 12
    assert lib.mrl_filter_doubles(_lib.ENV_CARTPOLE) == 2 + 2 * 5


def test_grids_sized_for_a_cu_subset():
    """desc.cus scales the grid caps (VF passes beside the rollout on 192 CUs): the VJP
    one block per CU, the row passes six; cus = 0 is the whole device (256)."""
    from modular_rl_amd import _lib
    lib = _lib.load()
    n = 4096 * 1024
    whole = _lib.MlpDesc(12, 1, _lib.HEAD_LINEAR, 64, 2)
    fit = _lib.MlpDesc(12, 1, _lib.HEAD_LINEAR, 64, 2, 192)
    for f, bf in [("mrl_mlp_slab_rows", "mrl_slab_rows"), ("mrl_mlp_partial_rows", "mrl_partial_rows"),
                  ("mrl_mlp_slab_rows_bf16", "mrl_slab_rows_bf16"),
                  ("mrl_mlp_partial_rows_bf16", "mrl_partial_rows_bf16")]:
        assert getattr(lib, f)(ctypes.byref(whole), n) == getattr(lib, bf)(n)
    assert lib.mrl_mlp_slab_rows(ctypes.byref(whole), n) == 256 * 4
    assert lib.mrl_mlp_slab_rows(ctypes.byref(fit), n) == 192 * 4
    assert lib.mrl_mlp_partial_rows(ctypes.byref(fit), n) == 6 * 192 * 4
    assert lib.mrl_mlp_slab_rows_bf16(ctypes.byref(fit), n) == 192 * 4
    assert lib.mrl_mlp_slab_rows(ctypes.byref(fit), 100) == 4  # small batches: one block
    bad = _lib.MlpDesc(12, 1, _lib.HEAD_LINEAR, 64, 2, -1)
    assert lib.mrl_mlp_slab_rows(ctypes.byref(bad), n) < 0


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU refusal")
def test_product_path_refuses_without_gpu():
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import MlpNet
    with pytest.raises(_lib.MrlError):
        MlpNet(11, 3, _lib.HEAD_GAUSS)


def test_hidden_sizes_validation_and_path_choice():
    from modular_rl_amd import _lib
    from modular_rl_amd.nets import check_hid_sizes, fused_ok
    assert check_hid_sizes([64, 64]) == [64, 64]
    assert check_hid_sizes(["512", 512, 512]) == [512, 512, 512]
    for bad in ([], [64, 0]):
        with pytest.raises(_lib.MrlError):
            check_hid_sizes(bad)
    assert fused_ok(11, 3, [64, 64]) and fused_ok(4, 2, [64, 64])
    assert not fused_ok(376, 17, [512, 512, 512]) and not fused_ok(11, 3, [128, 128])
    assert not fused_ok(40, 3, [64, 64]) and not fused_ok(11, 9, [64, 64])


def test_layered_parameter_layout_matches_the_reference():
    """LayeredMlpNet offsets follow Keras trainable_weights order (W, b per layer, logstd),
    checked against the oracle's unflatten without touching the GPU."""
    from modular_rl_amd.nets import layer_offsets
    from oracle import trpo_np as T
    for (nin, nout, name, hid) in [(376, 17, "gauss", [512, 512, 512]), (377, 1, "linear", [512, 512, 512]),
                                   (6, 5, "softmax", [100, 50, 30])]:
        spec = T.Spec(nin, hid, nout, name)
        dims = [nin] + hid + [nout]
        w_off, b_off, tls, P = layer_offsets(dims, name == "gauss")
        assert P == spec.P
        th = np.arange(spec.P, dtype=np.float64)
        Ws, bs, logstd = spec.split(th)
        for l in range(len(dims) - 1):
            assert Ws[l].shape == (dims[l], dims[l + 1])
            assert Ws[l].ravel()[0] == w_off[l] and bs[l].ravel()[0] == b_off[l]
        if name == "gauss":
            assert logstd.ravel()[0] == tls
    # Humanoid policy 376-512-512-512-17 (+logstd): SURVEY §8 C5
    assert T.Spec(376, [512, 512, 512], 17, "gauss").P == 376 * 512 + 512 + 2 * (512 * 512 + 512) + 512 * 17 + 17 + 17


def test_gemm_refuses_bad_descriptors():
    from modular_rl_amd import _lib
    lib = _lib.load()
    d = _lib.GemmDesc(m=4, n=4, k=4)
    rc = lib.mrl_gemm(ctypes.byref(d), None, None)
    assert rc < 0 and b"null" in lib.mrl_last_error()
    assert lib.mrl_gemm_slab_splits(1000, 4) == 4 and lib.mrl_gemm_slab_splits(10, 64) == 1
    # the column-tile choice (host query): 128-wide tiles from 160 blocks of 128x128 up
    tile = lambda **kw: lib.mrl_gemm_tile_n(ctypes.byref(_lib.GemmDesc(**kw)))
    assert tile(m=0, n=4, k=4) == 0 and lib.mrl_gemm_tile_n(None) == 0
    assert tile(m=1024, n=512, k=512) == 32          # 32 blocks: small-M launch
    assert tile(m=8192, n=512, k=512) == 128         # 256 blocks: the C5 layers' production tile
    assert tile(m=8192, n=17, k=512) == 32           # head layer
    assert tile(m=513, n=512, k=65536, epilogue=_lib.GEMM_SLAB, splits=64) == 128   # TN weight grads
    assert tile(m=513, n=512, k=65536, epilogue=_lib.GEMM_SLAB, splits=4) == 32


_UBSAN_PROBE = r"""
import ctypes, sys
from modular_rl_amd import _lib
lib = _lib.load()
# every status-returning entry point with null buffers: an error status, no fault
for name, (res, args) in _lib.SIGNATURES.items():
    if name in ("mrl_last_error", "mrl_version", "mrl_stream_destroy", "mrl_mlp_fisher_hyb_fits",
                "mrl_gemm_tile_n"):
        continue
    r = getattr(lib, name)(*[None if a is ctypes.c_void_p else 0 for a in args])
    if res is ctypes.c_int:
        assert r != 0, name
# the host-side sizing queries over valid and invalid descriptors and row counts
for n_in in (1, 4, 11, 16, 17, 32, 33):
    for n_out in (1, 2, 3, 8, 9):
        for head in (0, 1, 2):
            for hid in (64, 128):
                for cus in (0, 1, 64, 192, 256, 1024):
                    d = _lib.MlpDesc(n_in, n_out, head, hid, 2, cus)
                    b = ctypes.byref(d)
                    for f in ("mrl_mlp_num_params", "mrl_mlp_image_floats", "mrl_mlp_image_words_bf16",
                              "mrl_mlp_image_words_split", "mrl_mlp_fisher_hyb_fits"):
                        getattr(lib, f)(b)
                    for n in (0, 1, 31, 33, 4194304, 1 << 31):
                        lib.mrl_mlp_partial_rows(b, n); lib.mrl_mlp_slab_rows(b, n)
                        lib.mrl_mlp_partial_rows_bf16(b, n); lib.mrl_mlp_slab_rows_bf16(b, n)
for n in (0, 1, 31, 32, 33, 4194304, 1 << 31):
    lib.mrl_partial_rows(n); lib.mrl_slab_rows(n); lib.mrl_act_cache_floats(n); lib.mrl_act_cache_words_bf16(n)
    lib.mrl_cg_state_doubles(n); lib.mrl_moments_workspace_bytes(n); lib.mrl_episode_stats_workspace_bytes(n)
    lib.mrl_gae_workspace_bytes(n, 1024)
    for s in (1, 8, 64):
        lib.mrl_gemm_slab_splits(n, s)
        for m in (1, 513, 1 << 20):
            lib.mrl_gemm_tile_n(ctypes.byref(_lib.GemmDesc(m=m, n=512, k=n, epilogue=3, splits=s)))
for e in (-1, 0, 1, 2, 3, 99):
    lib.mrl_env_state_doubles(e); lib.mrl_filter_doubles(e); lib.mrl_record_doubles(e); lib.mrl_rollout_blocks(e)
print("UBSAN_PROBE_OK")
"""


def test_host_code_under_ubsan():
    """The C ABI's host code (argument checks, sizing queries, error paths) built with
    -fsanitize=undefined on the host side (`make ubsan`; -fno-sanitize-recover: any
    undefined behaviour aborts) and driven with null buffers and a sweep of valid and
    invalid descriptors in a child process -- no GPU needed."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "build", "ubsan", "libmrl_hip_ubsan.so")
    subprocess.run(["make", "-j8", "ubsan"], cwd=root, check=True, capture_output=True, timeout=900)
    env = dict(os.environ, MRL_LIB_PATH=so, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", _UBSAN_PROBE], cwd=root, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "UBSAN_PROBE_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]


def test_built_code_has_no_packed_f32_to_lds_reads():
    """The gfx950 code objects in libmrl_hip.so: no cross-lane LDS read (ds_bpermute /
    ds_permute / ds_swizzle) of a VGPR a packed-f32 VALU op wrote earlier in the same basic
    block, and no other LDS data read of one within 8 wait states (four times the count
    proven insufficient; the round-4 split Fisher product's run-to-run hazard).  A compiler or flag change that
    reintroduces the pattern fails here, on the CPU, before any GPU run."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_hazard_check as H
    lib = os.path.join(ROOT, "modular_rl_amd", "libmrl_hip.so")
    cos = H.code_objects(lib)
    assert len(cos) >= 7  # one per HIP source of the library
    bad = []
    for co in cos:
        bad += H.scan(H.disassemble(co))
    assert not bad, bad[:5]
    # and the checker does see the pattern: a packed-f32 sum read by ds_bpermute next
    lines = ["0000 <k>:", "v_pk_add_f32 v[4:5], v[0:1], v[34:35]", "v_add_f32_e32 v3, v2, v3",
             "ds_bpermute_b32 v6, v56, v4", "ds_bpermute_b32 v7, v56, v5"]
    assert [(f, st) for f, _, _, st in H.scan(lines)] == [("k", 1), ("k", 2)]
    # the build proven bad: two wait states (s_nop 1) before the bpermute; and a cross-lane
    # read far down the same block -- both flagged (whole-block rule for permutes)
    far = ["v_mul_f32_e32 v9, v8, v8"] * 40
    lines = ["0000 <k>:", "v_pk_add_f32 v[4:5], v[0:1], v[34:35]", "s_nop 1", "ds_bpermute_b32 v6, v56, v4"]
    assert [st for _, _, _, st in H.scan(lines)] == [2]
    lines = ["0000 <k>:", "v_pk_add_f32 v[4:5], v[0:1], v[34:35]"] + far + ["ds_swizzle_b32 v6, v5 offset:0x1f"]
    assert [st for _, _, _, st in H.scan(lines)] == [40]
    # other LDS data reads: flagged under 8 wait states, not beyond; a branch ends the block
    pk = ["0000 <k>:", "v_pk_mul_f32 v[4:5], v[0:1], v[34:35]"]
    assert [st for _, _, _, st in H.scan(pk + ["s_nop 5", "ds_write_b32 v6, v5"])] == [6]
    assert H.scan(pk + far[:8] + ["ds_write_b32 v6, v5"]) == []
    assert H.scan(pk + far[:8] + ["ds_write_b32 v6, v5"], min_states=None) != []
    assert H.scan(pk + ["s_branch 4", "ds_bpermute_b32 v6, v56, v4"]) == []
    # an overwrite in between clears the register
    assert H.scan(pk + ["v_mov_b32_e32 v4, 0", "ds_bpermute_b32 v6, v56, v4"]) == []
