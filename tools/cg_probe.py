"""Time the conjugate-gradient loop's iteration at the Hopper C3 size (4,194,304 rows):
one-pass Fisher product + CG update in two launch layouts -- product, slab reduction,
CG update, tangent pack (four launches); the CG update packing the tangent (three,
mrl_cg_update_pack) -- HIP events on the launch stream over many iterations, no profiler.
(Round 5 also measured a two-launch form with the reduction inside the CG update:
1218 us, the same; not kept, profiles/r05w_cg_probe.txt.)
Also a chain of tiny kernels (pack launches) to show the per-launch cost of a dependent
launch on this runtime."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, ptr, stream  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402
from modular_rl_amd.trpo import HipTrpoOps  # noqa: E402

N = int(os.environ.get("MRL_PROBE_ROWS", 4194304))


def timed(fn, reps):
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


rng = np.random.default_rng(0)
net = MlpNet(11, 3, _lib.HEAD_GAUSS)
net.set_flat(glorot_init(rng, 11, 3, _lib.HEAD_GAUSS))
g = torch.Generator(device='cuda').manual_seed(0)


class B:
    pass


b = B()
b.obs = torch.randn(N, 11, device='cuda', generator=g)
b.n = N
b.act = torch.randn(N, 3, device='cuda', generator=g)
b.adv = torch.randn(N, device='cuda', generator=g)
b.prob = net.forward(b.obs, N).clone()
ops = HipTrpoOps(net)
ops.bind(b, 1.0 / N)
ops.surrgrad()
g64 = ops.g.double()


def layout(pack):
    ops.cg_pack = pack

    def it():
        # tol 0: CG never converges, so the flag never stops the loop
        ops.cg_update(ops.fvp(ops.p32, skip=ops.flag), 1e-3, 0.0)
    ops.cg_init(g64)
    return it


LAYOUTS = (("4 launches (pack, product, reduce, update)", False),
           ("3 launches (update packs)", True))
res = {name: [] for name, _ in LAYOUTS}
timed(layout(True), 50)  # clocks up
for rnd in range(4):  # rotated, so clock drift does not favour one layout
    for name, pack in LAYOUTS:
        res[name].append(timed(layout(pack), 8) * 1e3)  # CG stays finite over a few iterations
for name, _ in LAYOUTS:
    print(f"{name:45s} median {np.median(res[name]):8.1f} us per CG iteration  "
          f"({' '.join(f'{v:.1f}' for v in res[name])})", flush=True)

# the dependent-launch cost: a chain of tiny kernels
img = net.new_tangent_image()


def chain():
    for _ in range(100):
        call("mrl_mlp_pack_split", ctypes_desc, ptr(ops.p32), ptr(img), None, stream())


ctypes_desc = ctypes.byref(net.desc)
print(f"tiny dependent launches: {timed(chain, 5) * 1e3 / 100:.2f} us per launch", flush=True)
