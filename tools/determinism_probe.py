"""Run-to-run determinism of the Fisher-product row kernels at 4.19 M rows: the same
launch repeated on the same inputs must give the same bits.  Prints, per kernel, how
many ghead rows differ from the first run across the repeats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = 1 << 22
REPS = int(os.environ.get("REPS", 6))
for label, dtype, split in (("f32", "fp32", False), ("split", "fp32", True), ("bf16", "bf16", False)):
    os.environ["MRL_FISHER"] = "split" if split else "f32"
    rng = np.random.default_rng(0)
    net = MlpNet(11, 3, _lib.HEAD_GAUSS, dtype=dtype)
    net.set_flat(glorot_init(rng, 11, 3, _lib.HEAD_GAUSS))
    torch.manual_seed(0)
    x = torch.randn(N, 11, device='cuda')
    act = torch.randn(N, 3, device='cuda')
    adv = torch.randn(N, device='cuda')
    prob = net.forward(x, N).clone()
    gh = torch.zeros(N * net.gh, device='cuda')
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    v = torch.randn(net.P, device='cuda') * 1e-2
    imgt = net.new_tangent_image()
    net.pack_tangent(v, imgt)
    net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh, partial=partial)
    outs = []
    for r in range(REPS):
        g = torch.zeros_like(gh)
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=g, tangent=v, image_t=imgt)
        outs.append(g.view(N, -1).cpu().numpy())
    bad = [int((o != outs[0]).any(1).sum()) for o in outs[1:]]
    cols = [np.nonzero((o != outs[0]).any(0))[0].tolist() for o in outs[1:]]
    print(f"{label}: rows differing from run 0 over {REPS - 1} repeats: {bad} cols {cols}", flush=True)
