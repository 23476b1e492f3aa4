"""Run-to-run determinism of the update's row / VJP kernels at 4.19 M rows (Hopper
policy): every launch repeated on the same inputs must give the same bits.  Prints per
kernel the number of output elements that differ from the first run over the repeats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = int(os.environ.get("MRL_PROBE_ROWS", 1 << 22))
REPS = int(os.environ.get("REPS", 4))


def check(label, fn):
    outs = [fn().cpu().numpy().copy() for _ in range(REPS)]
    bad = [int((o != outs[0]).sum()) for o in outs[1:]]
    print(f"{label}: elements differing from run 0: {bad}", flush=True)


for label, dtype, split, vsplit in (("f32", "fp32", False, False), ("split", "fp32", True, True),
                                    ("bf16", "bf16", False, False)):
    os.environ["MRL_FISHER"] = "split" if split else "f32"
    os.environ["MRL_VJP_SPLIT"] = "1" if vsplit else "0"
    rng = np.random.default_rng(0)
    net = MlpNet(11, 3, _lib.HEAD_GAUSS, dtype=dtype)
    net.set_flat(glorot_init(rng, 11, 3, _lib.HEAD_GAUSS))
    torch.manual_seed(0)
    x = torch.randn(N, 11, device='cuda')
    act = torch.randn(N, 3, device='cuda')
    adv = torch.randn(N, device='cuda')
    prob = net.forward(x, N).clone()
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    gh = torch.zeros(N * net.gh, device='cuda')
    v = torch.randn(net.P, device='cuda') * 1e-2
    imgt = net.new_tangent_image()
    net.pack_tangent(v, imgt)
    g = torch.zeros(net.P, device='cuda')

    def surrgrad():
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh,
                 partial=partial)
        return torch.cat([gh, partial.float()])

    def losses():
        net.rows(_lib.EPI_LOSSES, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, partial=partial,
                 theta=net.theta, image=net.image)
        return partial.clone()

    def fvp_rows():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgt)
        return gh.clone()

    def vjp():
        net.vjp_flat(x, N, gh, g)
        return g.clone()

    check(f"{label} prob", lambda: net.forward(x, N))
    check(f"{label} losses", losses)
    check(f"{label} surrgrad", surrgrad)
    check(f"{label} vjp(pg)", vjp)
    check(f"{label} fvp rows", fvp_rows)
    check(f"{label} vjp(fvp)", vjp)
