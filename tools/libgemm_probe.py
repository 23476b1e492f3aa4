"""Headroom probe: the vendor GEMM (torch.matmul -> hipBLASLt / rocBLAS) on the C5 layered
shapes (1,048,576 x 512 x 512 NN / NT / TN, bf16 and f32), against which this repo's
hand-written GEMMs (gemm.hip, gemm_bf16.hip) are compared.  Measurement only: the library
is not on the product path."""
import torch

M, N, K = 1048576, 512, 512


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


for dt in (torch.bfloat16, torch.float32):
    A = torch.randn(M, K, device="cuda", dtype=dt)
    W = torch.randn(K, N, device="cuda", dtype=dt)
    G = torch.randn(M, N, device="cuda", dtype=dt)
    fl = 2.0 * M * N * K
    for name, fn in (("NN  A.W", lambda: A @ W), ("NT  G.W^T", lambda: G @ W.t()), ("TN  A^T.G", lambda: A.t() @ G)):
        ms = timed(fn)
        print(f"{str(dt):15s} {name:10s} {ms:7.3f} ms  {fl / ms / 1e9:8.1f} TFLOP/s", flush=True)
    del A, W, G
    torch.cuda.empty_cache()
