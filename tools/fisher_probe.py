"""Time one Fisher product at the Hopper C3 size (4,194,304 rows) on the default paths:
the one-pass kernel (mrl_mlp_fisher_hyb) against the two-kernel pair (split JVP rows +
hybrid VJP), each with its slab reduction; HIP events on the launch stream.  Prints ms per
product and the max relative difference of the two products."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = int(os.environ.get("MRL_PROBE_ROWS", 4194304))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for nin, nout, head in ((11, 3, _lib.HEAD_GAUSS), (4, 2, _lib.HEAD_SOFTMAX)):
    rng = np.random.default_rng(0)
    net = MlpNet(nin, nout, head)
    net.set_flat(glorot_init(rng, nin, nout, head))
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn(N, nin, device='cuda', generator=g)
    act = (torch.randn(N, nout, device='cuda', generator=g) if head == _lib.HEAD_GAUSS
           else torch.randint(0, nout, (N,), device='cuda', dtype=torch.int32, generator=g))
    adv = torch.randn(N, device='cuda', generator=g)
    prob = net.forward(x, N).clone()
    gh = torch.zeros(N * net.gh, device='cuda')
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh, partial=partial)
    v = torch.randn(net.P, device='cuda', generator=g) * 1e-2
    imgs = net.new_tangent_image()
    net.pack_tangent(v, imgs)
    f1 = torch.zeros(net.P, device='cuda')
    f2 = torch.zeros(net.P, device='cuda')

    def onepass():
        assert net.fisher_product(x, N, 1.0 / N, v, imgs, f1)

    def twopass():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgs)
        net.vjp_flat(x, N, gh, f2)

    def jvp():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgs)

    def vjp():
        net.vjp_flat(x, N, gh, f2)

    t1, t2, tj, tv = timed(onepass), timed(twopass), timed(jvp), timed(vjp)
    rel = float((f1 - f2).abs().max() / f2.abs().max())
    print(f"[{nin},{nout},{head}] fisher product (+reduce): one-pass {t1:.4f} ms | two-pass {t2:.4f} ms "
          f"(JVP rows {tj:.4f} + VJP {tv:.4f}) | rel diff {rel:.3e}", flush=True)
