"""Diagnostic: which part of the process makes a rocprofv3-profiled run crash at exit.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/teardown_probe.py MODE
MODE: torch | lib (our kernels) | stream (+ CU-masked streams) | graph (+ a captured graph)
"""
import sys

import torch

sys.path.insert(0, '.')
mode = sys.argv[1]
x = torch.ones(1 << 20, device="cuda")
print("torch", float(x.sum()))
if mode in ("lib", "stream", "graph"):
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, ptr, stream
    _lib.load(require_gpu=True)
    T, E = 64, 256
    rew = torch.rand(T * E, device="cuda")
    v = torch.randn(T * E, device="cuda")
    flags = torch.zeros(T * E, dtype=torch.uint8, device="cuda")
    adv, ret = torch.empty_like(rew), torch.empty_like(rew)
    mom = torch.zeros(3, dtype=torch.float64, device="cuda")
    ws = torch.zeros(int(_lib.load().mrl_gae_workspace_bytes(T, E)), dtype=torch.uint8, device="cuda")

    def run():
        call("mrl_gae", ptr(rew), ptr(v), ptr(flags), T, E, 0.995, 0.97, ptr(adv), ptr(ret), ptr(mom), ptr(ws), stream())
    run()
    torch.cuda.synchronize()
    print("lib ok", float(mom[0]))
    if mode in ("stream", "graph"):
        from modular_rl_amd import streams
        s = streams.masked_stream(range(0, 64))
        with torch.cuda.stream(s):
            run()
        torch.cuda.synchronize()
        print("stream ok")
    if mode == "graph":
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g):
                run()
        g.replay()
        torch.cuda.synchronize()
        print("graph ok")
