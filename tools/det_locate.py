"""Locate the split Fisher-product rows' run-to-run differences (diagnostic).

Runs the split JVP rows kernel (mrl_mlp_fvp_split) REPS times on the same inputs at
4.19 M Hopper rows and, for every output element that differs between runs, reports
where it sits (row mod 64 -> lane quarter, tile) and what the odd value equals: the
majority value of another row / column of the same tile, the value before the final
scaling, etc.  MRL_LIB_PATH selects the library build under test."""
import os
import sys
from collections import Counter

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = int(os.environ.get("MRL_PROBE_ROWS", 1 << 22))
REPS = int(os.environ.get("REPS", 6))
os.environ["MRL_FISHER"] = "split"
rng = np.random.default_rng(0)
net = MlpNet(11, 3, _lib.HEAD_GAUSS, dtype="fp32")
th = glorot_init(rng, 11, 3, _lib.HEAD_GAUSS)
net.set_flat(th)
torch.manual_seed(0)
x = torch.randn(N, 11, device='cuda')
act = torch.randn(N, 3, device='cuda')
adv = torch.randn(N, device='cuda')
prob = net.forward(x, N).clone()
partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
gh = torch.zeros(N * net.gh, device='cuda')
net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh, partial=partial)
v = torch.randn(net.P, device='cuda') * 1e-2
imgt = net.new_tangent_image()
net.pack_tangent(v, imgt)
outs = []
for _ in range(REPS):
    gh.zero_()
    net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgt)
    outs.append(gh.view(N, net.gh).cpu().numpy().copy())
torch.cuda.synchronize()
O = np.stack(outs)  # [REPS, N, gh]
diff = (O != O[0:1]).any(axis=0)
print(f"lib={_lib.LIB_PATH} rows={N} reps={REPS} differing elements={int(diff.sum())} "
      f"rows={int(diff.any(axis=1).sum())} cols={sorted(set(np.nonzero(diff)[1].tolist()))}", flush=True)
if diff.any():
    # majority value per element
    rows, cols = np.nonzero(diff)
    good = np.empty(len(rows), np.float32)
    for i, (r, c) in enumerate(zip(rows, cols)):
        good[i] = Counter(O[:, r, c].tolist()).most_common(1)[0][0]
    lanes = rows % 32
    print("row mod 32 histogram:", np.bincount(lanes, minlength=32).tolist())
    print("quarter (row%32)//16:", np.bincount(lanes // 16, minlength=2).tolist(),
          " tile%4 (wave in block):", np.bincount((rows // 32) % 4, minlength=4).tolist())
    groups = sorted(set((rows // 16).tolist()))
    print("16-row groups:", len(groups), "first:", groups[:12])
    ls = th[-3:]
    var = np.exp(2 * ls).astype(np.float32)
    shown = 0
    for i, (r, c) in enumerate(zip(rows, cols)):
        vals = O[:, r, c]
        bad = [b for b in vals if b != good[i]]
        if not bad or shown >= 12:
            continue
        b = bad[0]
        t0 = (r // 32) * 32
        tile_good = np.array([Counter(O[:, rr, c].tolist()).most_common(1)[0][0] for rr in range(t0, t0 + 32)])
        same_row_other = [cc for cc in range(net.gh) if cc != c and O[0, r, cc] == b]
        other_rows = [int(t0 + k) for k in np.nonzero(tile_good == b)[0]]
        print(f"  row {r} (tile {r // 32}, lane {r % 32}) col {c}: good {good[i]:.9g} bad {b:.9g} "
              f"ratio {b / good[i]:.6g} good*var {good[i] * var[c] * N:.6g} bad*var*N {b * var[c] * N:.6g} "
              f"same-row cols {same_row_other} rows-in-tile {other_rows}", flush=True)
        shown += 1
