"""Diagnostic: where the split FVP rows differ from the exact-f32 kernel's (Hopper shape)."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

for N in (3001, 65536, 1 << 22):
    rng = np.random.default_rng(0)
    nin, nout, head = 11, 3, _lib.HEAD_GAUSS
    net = MlpNet(nin, nout, head)
    net.set_flat(glorot_init(rng, nin, nout, head))
    torch.manual_seed(0)
    x = torch.randn(N, nin, device='cuda')
    act = torch.randn(N, nout, device='cuda')
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
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=img32)
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh_s, tangent=v, image_t=imgs)
    a, b = gh.view(N, -1).cpu().numpy(), gh_s.view(N, -1).cpu().numpy()
    d = np.abs(a - b)
    r, c = np.unravel_index(np.argmax(d), d.shape)
    big = (d > 1e-4 * np.abs(a).max()).any(1)
    print(f"N={N}: max diff {d.max():.3e} at row {r} col {c} (f32 {a[r, c]:.6e} split {b[r, c]:.6e}), "
          f"max|a| {np.abs(a).max():.3e}; rows with diff > 1e-4 max: {big.sum()} first {np.nonzero(big)[0][:10]} "
          f"tile {r // 32} lane-row {r % 32}; xnorm {float(x[r].abs().max()):.3f}", flush=True)
    if big.sum():
        rows = np.nonzero(big)[0][:5]
        print("  f32  :", a[rows][:, :3], "\n  split:", b[rows][:, :3], flush=True)
        # float64 truth of the mean-head rows: central differences of the oracle forward
        sys.path.insert(0, '.')
        from oracle import trpo_np as T
        spec = T.Spec(nin, [64, 64], nout, "gauss")
        th = net.theta.double().cpu().numpy()
        vv = v.double().cpu().numpy()
        xr = x[rows].double().cpu().numpy()
        eps = 1e-3
        mp = T.policy_prob(spec, th + eps * vv, xr)[:, :nout]
        mm = T.policy_prob(spec, th - eps * vv, xr)[:, :nout]
        sd = np.exp(th[-nout:])
        want = (mp - mm) / (2 * eps) / sd ** 2 / N
        print("  f64  :", want, flush=True)
