"""Run ONE layered-path GEMM shape repeatedly, for rocprofv3 counter passes over it.

    python tools/gemm_pmc_probe.py gemm:bf16:NN_dual_dtanh:1048576x512x512 [reps]

The label is the one bench.py's roofline_policy_gemm names (the timing region of
modular_rl_amd/nets.py: dtype, kind, m x n x k).  The operands are built and cast first
(cast / pack kernels; tools/pmc_traffic.py --gemm ignores them), then the GEMM runs
`reps` times on the same operands, as in a Fisher product."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
label = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
_, dt, kind, shape = label.split(":")
m, n, k = (int(v) for v in shape.split("x"))
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
ld8 = lambda d: (d + 7) // 8 * 8  # noqa: E731


def bf16_rows(rows, cols, ld, scale=1.0):
    x = torch.randn(rows * cols, device="cuda") * scale
    y = torch.zeros(rows * ld, dtype=torch.int16, device="cuda")
    call("mrl_cast_rows_bf16", P(x), rows, cols, cols, P(y), ld, stream())
    return y


if dt == "bf16" and kind == "TN":
    # weight gradient over k rows: a [k, m-1 (+ ones column)], b [k, n]
    din = m - 1
    A, B = bf16_rows(k, din, ld8(din)), bf16_rows(k, n, ld8(n))
    S = int(lib.mrl_gemm_slab_splits(k, 64))
    slab = torch.empty(S * m * n, device="cuda")
    g = _lib.GemmBf16TnDesc(m=m, n=n, k=k, a=P(A), lda=ld8(din), b=P(B), ldb=ld8(n), ones_row=1, splits=64,
                            slab=P(slab), slab_stride=m * n, ldc=n)
    run = lambda: call("mrl_gemm_bf16_tn", ctypes.byref(g), None, stream())  # noqa: E731
elif dt == "bf16":
    dual = "dual" in kind
    epi = _lib.GEMM_TANH if kind.endswith("_tanh") else (_lib.GEMM_DTANH if kind.endswith("_dtanh") else
                                                         _lib.GEMM_STORE)
    A = bf16_rows(m, k, ld8(k))
    W = torch.randn(k * n, device="cuda") * 0.05
    Bt = torch.zeros(n * ld8(k), dtype=torch.int16, device="cuda")
    call("mrl_pack_w_bf16", P(W), k, n, 1, P(Bt), ld8(k), stream())
    H = bf16_rows(m, n, n, 0.5) if epi == _lib.GEMM_DTANH else None
    c_bf16 = epi != _lib.GEMM_STORE
    C = torch.empty(m * n, dtype=torch.int16 if c_bf16 else torch.float32, device="cuda")
    bias = torch.zeros(n, device="cuda")
    g = _lib.GemmBf16Desc(m=m, n=n, k=k, a=P(A), lda=ld8(k), bt=P(Bt), ldb=ld8(k), a2=P(A) if dual else None,
                          bt2=P(Bt) if dual else None, c=P(C), ldc=n, c_bf16=int(c_bf16), epilogue=epi, bias=P(bias),
                          h=P(H) if H is not None else None, ldh=n)
    run = lambda: call("mrl_gemm_bf16", ctypes.byref(g), None, stream())  # noqa: E731
else:
    raise SystemExit(f"{label}: only the bf16 layered GEMMs are probed")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
print(f"{label}: {e0.elapsed_time(e1) / reps:.4f} ms per launch over {reps}", flush=True)
