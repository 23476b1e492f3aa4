"""Diagnostic: the bf16 TN weight-gradient GEMM at the Humanoid layer shape (K = 1,048,576
rows, 512 (+ ones row) x 512, 64 split-K slabs): 128 x 128 tiled kernel vs the 256 x 256
LDS-DMA kernel (+ bias column sum), ms per launch and TFLOP/s (algorithmic 2 M N K)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
R = 1 << 20
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for din, dout, ones in [(512, 512, True), (376, 512, True), (512, 512, False)]:
    lda = (din + 7) // 8 * 8
    X = (torch.randn(R * lda, device="cuda") * 0.5).to(torch.bfloat16).view(torch.int16)
    G = (torch.randn(R * dout, device="cuda") * 0.5).to(torch.bfloat16).view(torch.int16)
    M = din + int(ones)
    S = int(lib.mrl_gemm_slab_splits(R, 64))
    slab = torch.zeros(S * M * dout, dtype=torch.float32, device="cuda")
    g = _lib.GemmBf16TnDesc(m=M, n=dout, k=R, a=P(X), lda=lda, b=P(G), ldb=dout, ones_row=int(ones), splits=64,
                            slab=P(slab), slab_stride=M * dout, ldc=dout)
    res = []
    for name, big in (("tiled128", "0"), ("big256", "1")):
        os.environ["MRL_GEMM_TN_BIG"] = big
        t = timed(lambda: call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream()))
        res.append(f"{name} {t:.3f} ms {2.0 * M * dout * R / t / 1e9:.0f} TF")
    print(f"TN rows={R} {M}x{dout} ones={ones}: " + " | ".join(res), flush=True)
