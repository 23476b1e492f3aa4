"""Time the Hopper-shaped Fisher-product kernels (FVP JVP rows with the activation
cache + the cached VJP) and the loss passes at 4.19 M rows; MRL_LIB_PATH selects an
ablation build (tools/build_ablate.sh)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = 4194304
rng = np.random.default_rng(0)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    # MRL_PROBE_NET=nin,nout,head (head gauss | softmax), default the Hopper policy 11,3,gauss
    nin, nout, hname = (os.environ.get("MRL_PROBE_NET") or "11,3,gauss").split(",")
    nin, nout = int(nin), int(nout)
    head = _lib.HEAD_GAUSS if hname == "gauss" else _lib.HEAD_SOFTMAX
    net = MlpNet(nin, nout, head, dtype=os.environ.get("MRL_PROBE_DTYPE", "fp32"))
    net.set_flat(glorot_init(rng, nin, nout, head))
    x = torch.randn(N, nin, device='cuda')
    act = (torch.randn(N, nout, device='cuda') if head == _lib.HEAD_GAUSS
           else torch.randint(0, nout, (N,), device='cuda', dtype=torch.int32))
    adv = torch.randn(N, device='cuda')
    prob = net.forward(x, N).clone()
    gh = torch.zeros(N * net.gh, device='cuda')
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device='cuda')
    g = torch.zeros(net.P, device='cuda')
    v = torch.randn(net.P, device='cuda') * 1e-2
    imgt = torch.zeros_like(net.image)
    net.pack(theta=v, image=imgt, fwd_only=True)

    def surrgrad():
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=gh,
                 partial=partial)

    def jvp():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=gh, tangent=v, image_t=imgt)

    def vjp():
        net.vjp_flat(x, N, gh, g)

    def prob_pass():
        net.forward(x, N, out=prob)

    lib = os.environ.get("MRL_LIB_PATH", "default")
    surrgrad()
    print(f"[{os.path.basename(lib)} {net.dtype} {nin},{nout},{hname}] surrgrad {timed(surrgrad):.3f} ms  "
          f"fvp_jvp_rows {timed(jvp):.3f} ms  vjp {timed(vjp):.3f} ms  prob {timed(prob_pass):.3f} ms", flush=True)
    # the same Fisher-product pair recomputing the primal activations (no cache reads)
    net.use_cache = False
    print(f"[{os.path.basename(lib)} {net.dtype} {nin},{nout},{hname}] uncached: fvp_jvp_rows {timed(jvp):.3f} ms  "
          f"vjp {timed(vjp):.3f} ms", flush=True)
    net.use_cache = True


if __name__ == "__main__":
    main()
