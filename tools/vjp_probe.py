"""Time the fused VJP kernel (cached / uncached) for policy- and VF-shaped nets."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402
N = 4194304
rng = np.random.default_rng(0)


def run(nin, nout, head, ept_kind):
    net = MlpNet(nin, nout, head)
    net.set_flat(glorot_init(rng, nin, nout, head))
    nobs = nin - 1 if ept_kind else nin
    x = torch.randn(N, nobs, device='cuda')
    ept = None
    if ept_kind == "zero":
        ept = torch.zeros(N, dtype=torch.int32, device='cuda')
    elif ept_kind == "rand":
        ept = torch.randint(0, 1000, (N,), dtype=torch.int32, device='cuda')
    lim = 1000.0
    gh = torch.randn(N * net.gh, device='cuda') * 1e-3
    g = torch.zeros(net.P, device='cuda')
    tgt = torch.randn(N, device='cuda')
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    if head == _lib.HEAD_LINEAR:
        net.rows(_lib.EPI_VFLOSS, x, N, ep_t=ept, timestep_limit=lim, inv_n_global=1.0 / N, target=tgt, ghead=gh,
                 partial=partial)
    else:
        act = torch.randn(N, nout, device='cuda')
        adv = torch.randn(N, device='cuda')
        prob = net.forward(x, N).clone()
        net.rows(_lib.EPI_SURRGRAD, x, N, timestep_limit=lim, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob,
                 ghead=gh, partial=partial)
    for cache in (True, False):
        net.use_cache = cache
        net.vjp_flat(x, N, gh, g, ep_t=ept, timestep_limit=lim)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            net.vjp_flat(x, N, gh, g, ep_t=ept, timestep_limit=lim)
        e1.record()
        torch.cuda.synchronize()
        print(f"nin={nin} nout={nout} head={head} ept={ept_kind} cache={cache}: {e0.elapsed_time(e1) / 5:.3f} ms",
              flush=True)
        net.use_cache = True


run(11, 3, _lib.HEAD_GAUSS, None)
run(12, 1, _lib.HEAD_LINEAR, "rand")
run(12, 1, _lib.HEAD_LINEAR, "zero")
run(12, 1, _lib.HEAD_LINEAR, None)
run(11, 1, _lib.HEAD_LINEAR, None)
