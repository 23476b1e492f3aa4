"""Diagnostic: the 256 x 256 bf16 NN kernel alone at M = 1,048,576, K = N = 512, per
epilogue (tanh / plain store, bf16 out).  Run once with the production library and once
with MRL_LIB_PATH=tools/ablate/libmrl_hip_noepi.so (tools/build_ablate.sh noepi
-DMRL_BIG_ABL_NOEPI) to split the K loop from the epilogue."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
M = 1 << 20
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
os.environ["MRL_GEMM_BIG_MIN_M"] = "1"


def timed(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tag = os.environ.get("MRL_LIB_PATH", "production")
for (K, N, dual, epi, outbf, bias) in [(512, 512, False, _lib.GEMM_TANH, 1, True),
                                       (512, 512, False, _lib.GEMM_TANH, 1, False),
                                       (512, 512, False, _lib.GEMM_STORE, 1, True),
                                       (512, 512, True, _lib.GEMM_DTANH, 1, True)]:
    flop = 2.0 * M * N * K * (2 if dual else 1)
    Ab = (torch.randn(M * K, device="cuda") * 0.5).to(torch.bfloat16).view(torch.int16)
    Hb = (torch.rand(M * N, device="cuda") * 0.9).to(torch.bfloat16).view(torch.int16)
    W = torch.randn(K * N, device="cuda") * 0.05
    Bt = torch.zeros(N * K, dtype=torch.int16, device="cuda")
    call("mrl_pack_w_bf16", P(W), K, N, 1, P(Bt), K, stream())
    Cb = torch.empty(M * N, dtype=torch.int16, device="cuda")
    bv = torch.randn(N, device="cuda") * 0.1
    gb = _lib.GemmBf16Desc(m=M, n=N, k=K, a=P(Ab), lda=K, bt=P(Bt), ldb=K, a2=P(Ab) if dual else None,
                           bt2=P(Bt) if dual else None, c=P(Cb), ldc=N, c_bf16=outbf, epilogue=epi, h=P(Hb), ldh=N,
                           bias=P(bv) if bias else None)
    t = timed(lambda: call("mrl_gemm_bf16", ctypes.byref(gb), None, stream()))
    print(f"{tag} NN K={K} N={N} dual={dual} epi={epi} bias={bias}: {t:.3f} ms {flop / t / 1e9:.0f} TF",
          flush=True)
