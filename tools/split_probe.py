"""Time and compare the Fisher product's JVP half at 4.19 M rows: the exact-f32 kernel
(mlp_rows_kernel<EPI_FVP_CACHED>) against the split-operand bf16 kernel
(mlp_fvp_split_kernel), both reading the f32 activation cache of one SURRGRAD pass;
prints ms per launch and the max relative difference of the head-gradient rows and of
the whole Fisher product (the same cached VJP of each)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = int(os.environ.get("MRL_PROBE_ROWS", 4194304))


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


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


CASES = ((11, 3, _lib.HEAD_GAUSS), (4, 2, _lib.HEAD_SOFTMAX))
for nin, nout, head in CASES[:int(os.environ.get("MRL_PROBE_NCASES", len(CASES)))]:  # 1: Hopper's net only
    rng = np.random.default_rng(0)
    net = MlpNet(nin, nout, head)
    net.set_flat(glorot_init(rng, nin, nout, head))
    x = torch.randn(N, nin, device='cuda')
    act = (torch.randn(N, nout, device='cuda') if head == _lib.HEAD_GAUSS
           else torch.randint(0, nout, (N,), device='cuda', dtype=torch.int32))
    adv = torch.randn(N, device='cuda')
    prob = net.forward(x, N).clone()
    gh = torch.zeros(N * net.gh, device='cuda')
    gh_s = torch.zeros_like(gh)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    v = torch.randn(net.P, device='cuda') * 1e-2
    img32 = torch.zeros_like(net.image)
    net.pack(theta=v, image=img32, fwd_only=True)
    imgs = net.new_tangent_image()
    net.pack_tangent(v, imgs)
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh, partial=partial)

    def jvp32():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=img32)

    def jvps():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh_s, tangent=v, image_t=imgs)

    t32, ts = timed(jvp32), timed(jvps)
    f32 = torch.zeros(net.P, device='cuda')
    fs = torch.zeros(net.P, device='cuda')
    tv = timed(lambda: net.vjp_flat(x, N, gh, f32))  # the cached VJP (mlp_vjp16_kernel, hybrid)
    net.vjp_flat(x, N, gh_s, fs)
    torch.cuda.synchronize()
    print(f"[{nin},{nout},{head}] fvp rows: f32 {t32:.4f} ms  split {ts:.4f} ms | vjp(+reduce) {tv:.4f} ms | "
          f"ghead rel diff {rel(gh_s, gh):.3e}  Fv (split rows vs f32 rows) rel diff {rel(fs, f32):.3e}", flush=True)
