"""Diagnostic: the 256 x 256 LDS-DMA and streaming bf16 NN kernels vs the tiled one at the Humanoid layer shapes
(M = 1,048,576 rows): ms per launch, TFLOP/s, and algorithmic HBM GB/s (A + A2 read once,
C and H once; Bt from L2)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
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


for (K, N, dual, epi, outbf) in [(512, 512, False, _lib.GEMM_TANH, 1), (512, 512, True, _lib.GEMM_DTANH, 1),
                                 (376, 512, False, _lib.GEMM_TANH, 1), (512, 512, False, _lib.GEMM_DTANH, 1),
                                 (512, 512, False, _lib.GEMM_STORE, 0)]:
    ldk = (K + 7) // 8 * 8
    flop = 2.0 * M * N * K * (2 if dual else 1)
    byts = M * ldk * 2 * (2 if dual else 1) + M * N * (2 if outbf else 4) + (M * N * 2 if epi == _lib.GEMM_DTANH else 0)
    # finite bf16 operands (random int16 bit patterns hold NaNs, whose payloads need not agree)
    Ab = (torch.randn(M * ldk, device="cuda") * 0.5).to(torch.bfloat16).view(torch.int16)
    Hb = (torch.rand(M * N, device="cuda") * 1.8 - 0.9).to(torch.bfloat16).view(torch.int16)
    W = torch.randn(K * N, device="cuda") * 0.05
    Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
    call("mrl_pack_w_bf16", P(W), K, N, 1, P(Bt), ldk, stream())
    Cb = torch.empty(M * N, dtype=torch.int16 if outbf else torch.float32, device="cuda")
    gb = _lib.GemmBf16Desc(m=M, n=N, k=K, a=P(Ab), lda=ldk, bt=P(Bt), ldb=ldk, a2=P(Ab) if dual else None,
                           bt2=P(Bt) if dual else None, c=P(Cb), ldc=N, c_bf16=outbf, epilogue=epi, h=P(Hb), ldh=N)
    res = []
    outs = []
    for name, big, mm in (("tiled", "0", "0"), ("stream", "0", "1"), ("big256", "1", "0")):
        os.environ["MRL_GEMM_BIG_MIN_M"] = big
        os.environ["MRL_GEMM_STREAM_MIN_M"] = mm
        t = timed(lambda: call("mrl_gemm_bf16", ctypes.byref(gb), None, stream()))
        outs.append(Cb.clone())
        res.append(f"{name} {t:.3f} ms {flop / t / 1e9:.0f} TF {byts / t / 1e6:.0f} GB/s")
    res.append("big==tiled" if torch.equal(outs[0], outs[2]) else "BIG DIFFERS")
    print(f"NN K={K} N={N} dual={dual} epi={epi} outbf={outbf}: " + " | ".join(res), flush=True)
