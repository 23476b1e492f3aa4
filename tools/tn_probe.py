"""Time the tiled bf16 TN GEMM (weight-gradient slabs) at C5 shapes, register stages
in flight 1 vs 4 (MRL_GEMM_TN_DEPTH): the policy head layer 513 x 17 over 1 M rows and
the VF input layer 378 x 512 (377 rows + ones, the tiled kernel's case)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

R = 1048576
for din, dout in ((512, 17), (377, 512)):
    lda, ldb = (din + 7) // 8 * 8, (dout + 7) // 8 * 8
    X = torch.randint(-3000, 3000, (R * lda,), dtype=torch.int16, device="cuda") & 0x3FFF
    G = torch.randint(-3000, 3000, (R * ldb,), dtype=torch.int16, device="cuda") & 0x3FFF
    M = din + 1
    S = int(_lib.load().mrl_gemm_slab_splits(R, 64))
    slab = torch.zeros(S * M * dout, dtype=torch.float32, device="cuda")
    g = _lib.GemmBf16TnDesc(m=M, n=dout, k=R, a=ctypes.c_void_p(X.data_ptr()), lda=lda,
                            b=ctypes.c_void_p(G.data_ptr()), ldb=ldb, ones_row=1, splits=64,
                            slab=ctypes.c_void_p(slab.data_ptr()), slab_stride=M * dout, ldc=dout)
    os.environ["MRL_GEMM_TN_BIG"] = "0"
    for depth in ("1", "4"):
        os.environ["MRL_GEMM_TN_DEPTH"] = depth
        call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        gb = 2 * R * (lda + ldb) / 1e9
        print(f"TN {M}x{dout}x{R} depth {depth}: {ms:.4f} ms, {gb / ms:.2f} TB/s of operand reads", flush=True)
