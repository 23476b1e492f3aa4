"""Diagnostic: the layered-path GEMMs at the Humanoid shapes (M = 1,048,576 rows),
fp32-staged bf16 (mrl_gemm, MRL_COMPUTE_BF16) vs bf16-operand (mrl_gemm_bf16 /
mrl_gemm_bf16_tn): ms per launch and TFLOP/s."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for (K, N, dual, epi) in [(512, 512, False, _lib.GEMM_TANH), (512, 512, True, _lib.GEMM_DTANH), (376, 512, False, _lib.GEMM_DTANH),
                          (512, 17, True, _lib.GEMM_STORE)]:
    flop = 2.0 * M * N * K * (2 if dual else 1)
    A = torch.randn(M * K, device="cuda")
    W = torch.randn(K * N, device="cuda") * 0.05
    H = torch.tanh(torch.randn(M * N, device="cuda"))
    C = torch.empty(M * N, device="cuda")
    g = _lib.GemmDesc(m=M, n=N, k=K, a=P(A), lda=K, b=P(W), ldb=N, epilogue=epi, a2=P(A) if dual else None,
                      b2=P(W) if dual else None, c=P(C), ldc=N, h=P(H), ldh=N, compute=_lib.COMPUTE_BF16)
    t_old = timed(lambda: call("mrl_gemm", ctypes.byref(g), None, stream()))
    Ab = torch.empty(M * K, dtype=torch.int16, device="cuda")
    Hb = torch.empty(M * N, dtype=torch.int16, device="cuda")
    call("mrl_cast_rows_bf16", P(A), M, K, K, P(Ab), K, stream())
    call("mrl_cast_rows_bf16", P(H), M, N, N, P(Hb), N, stream())
    ldk = (K + 7) // 8 * 8
    Bt = torch.zeros(N * ldk, dtype=torch.int16, device="cuda")
    call("mrl_pack_w_bf16", P(W), K, N, 1, P(Bt), ldk, stream())
    Cb = torch.empty(M * N, dtype=torch.int16, device="cuda")
    gb = _lib.GemmBf16Desc(m=M, n=N, k=K, a=P(Ab), lda=K, bt=P(Bt), ldb=ldk, a2=P(Ab) if dual else None,
                           bt2=P(Bt) if dual else None, c=P(Cb), ldc=N, c_bf16=int(N > 32), epilogue=epi, h=P(Hb), ldh=N)
    t_new = timed(lambda: call("mrl_gemm_bf16", ctypes.byref(gb), None, stream()))
    print(f"NN K={K} N={N} dual={dual}: fp32-staged {t_old:.3f} ms {flop / t_old / 1e9:.0f} TF | bf16-operand "
          f"{t_new:.3f} ms {flop / t_new / 1e9:.0f} TF", flush=True)

# weight gradient TN: C[din+1][dout] over M rows
for (din, dout) in [(512, 512), (376, 512), (512, 17)]:
    flop = 2.0 * M * (din + 1) * dout
    X = torch.randn(M * din, device="cuda")
    G = torch.randn(M * dout, device="cuda")
    S = int(lib.mrl_gemm_slab_splits(M, 64))
    slab = torch.empty(S * (din + 1) * dout, device="cuda")
    g = _lib.GemmDesc(m=din + 1, n=dout, k=M, a=P(X), lda=din, a_trans=1, ones_row=1, b=P(G), ldb=dout,
                      epilogue=_lib.GEMM_SLAB, c=P(slab), ldc=dout, splits=64, slab_stride=(din + 1) * dout,
                      compute=_lib.COMPUTE_BF16)
    t_old = timed(lambda: call("mrl_gemm", ctypes.byref(g), None, stream()))
    ldx, ldg = (din + 7) // 8 * 8, (dout + 7) // 8 * 8
    Xb = torch.empty(M * ldx, dtype=torch.int16, device="cuda")
    Gb = torch.empty(M * ldg, dtype=torch.int16, device="cuda")
    call("mrl_cast_rows_bf16", P(X), M, din, din, P(Xb), ldx, stream())
    call("mrl_cast_rows_bf16", P(G), M, dout, dout, P(Gb), ldg, stream())
    gt = _lib.GemmBf16TnDesc(m=din + 1, n=dout, k=M, a=P(Xb), lda=ldx, b=P(Gb), ldb=ldg, ones_row=1, splits=64,
                             slab=P(slab), slab_stride=(din + 1) * dout, ldc=dout)
    t_new = timed(lambda: call("mrl_gemm_bf16_tn", ctypes.byref(gt), None, stream()))
    print(f"TN din={din} dout={dout}: fp32-staged {t_old:.3f} ms {flop / t_old / 1e9:.0f} TF | bf16-operand "
          f"{t_new:.3f} ms {flop / t_new / 1e9:.0f} TF", flush=True)
