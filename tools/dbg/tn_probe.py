"""Diagnostic: where single one-hot products land in mrl_gemm_bf16_tn."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, stream  # noqa: E402

lib = _lib.load(require_gpu=True)
R, din, dout = 32, 128, 128


def run(X, G):
    x = torch.tensor(X.astype(np.float32), device="cuda")
    g = torch.tensor(G.astype(np.float32), device="cuda")
    bx = torch.zeros(R * din, dtype=torch.int16, device="cuda")
    bg = torch.zeros(R * dout, dtype=torch.int16, device="cuda")
    call("mrl_cast_rows_bf16", ctypes.c_void_p(x.data_ptr()), R, din, din, ctypes.c_void_p(bx.data_ptr()), din, stream())
    call("mrl_cast_rows_bf16", ctypes.c_void_p(g.data_ptr()), R, dout, dout, ctypes.c_void_p(bg.data_ptr()), dout, stream())
    slab = torch.zeros(din * dout, dtype=torch.float32, device="cuda")
    d = _lib.GemmBf16TnDesc(m=din, n=dout, k=R, a=ctypes.c_void_p(bx.data_ptr()), lda=din, b=ctypes.c_void_p(bg.data_ptr()),
                            ldb=dout, ones_row=0, splits=1, slab=ctypes.c_void_p(slab.data_ptr()), slab_stride=0, ldc=dout)
    call("mrl_gemm_bf16_tn", ctypes.byref(d), None, stream())
    return slab.cpu().numpy().reshape(din, dout)


for (r0, i0, j0) in [(0, 0, 0), (1, 0, 0), (4, 0, 0), (8, 0, 0), (0, 1, 0), (0, 5, 0), (0, 17, 0), (0, 0, 1), (0, 0, 5),
                     (0, 0, 17), (0, 33, 40), (17, 3, 7)]:
    X = np.zeros((R, din)); G = np.zeros((R, dout))
    X[r0, i0] = 1; G[r0, j0] = 1
    C = run(X, G)
    nz = np.argwhere(C != 0)
    print((r0, i0, j0), "->", [tuple(v) + (float(C[tuple(v)]),) for v in nz[:6]], flush=True)
