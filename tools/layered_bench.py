"""Time the layered (GEMM) MLP passes on a Humanoid-shaped net: forward, surrogate
gradient (forward + VJP), Fisher product (JVP + VJP on the recorded tape), and the
value-net loss/grad.  Prints one JSON line per pass with ms and achieved TFLOP/s.

    python tools/layered_bench.py [--rows N] [--reps R]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd.nets import LayeredMlpNet, glorot_init  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--obs", type=int, default=376)
    ap.add_argument("--act", type=int, default=17)
    ap.add_argument("--hid", type=str, default="512,512,512")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    args = ap.parse_args()
    hid = [int(h) for h in args.hid.split(",")]
    N, O, A = args.rows, args.obs, args.act
    rng = np.random.default_rng(0)
    net = LayeredMlpNet(O, A, _lib.HEAD_GAUSS, hid, dtype=args.dtype)
    net.set_flat(glorot_init(rng, O, A, _lib.HEAD_GAUSS, hid))
    dev = "cuda"
    x = torch.randn(N, O, device=dev)
    act = torch.randn(N, A, device=dev)
    adv = torch.randn(N, device=dev)
    prob = net.forward(x, N).clone()
    ghead = torch.zeros(N * net.gh, device=dev)
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device=dev)
    g = torch.zeros(net.P, device=dev)
    v = torch.randn(net.P, device=dev) * 1e-2
    dims = [O] + hid + [A]
    fwd_flops = 2.0 * N * sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    def fwd():
        net.forward(x, N, out=prob)

    def surr():
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=adv, oldprob=prob, ghead=ghead,
                 partial=partial)
        net.vjp_flat(x, N, ghead, g)

    def fvp():
        net.rows(_lib.EPI_FVP, x, N, inv_n_global=1.0 / N, ghead=ghead, tangent=v)
        net.vjp_flat(x, N, ghead, g)

    surr()
    res = {}
    first = 2.0 * N * dims[0] * dims[1]  # layer 0 has no input grad and a single JVP product
    for name, fn, fl in [("forward", fwd, fwd_flops), ("surrgrad_fwd_vjp", surr, 3 * fwd_flops - first),
                         ("fvp_jvp_vjp", fvp, 4 * fwd_flops - 2 * first)]:
        ms = timed(fn)
        res[name] = ms
        print(json.dumps({"pass": name, "rows": N, "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
