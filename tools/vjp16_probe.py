"""Time the cached VJP kernel (mlp_vjp16_kernel, hybrid form) at the Hopper C3 size
(4,194,304 rows): the VJP launch alone (no slab reduction), HIP events on the launch
stream."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, ptr, stream  # noqa: E402
from modular_rl_amd.nets import MlpNet, glorot_init  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4194304
rng = np.random.default_rng(0)
for nin, nout, head in [(11, 3, _lib.HEAD_GAUSS), (4, 2, _lib.HEAD_SOFTMAX), (12, 1, _lib.HEAD_LINEAR)]:
    net = MlpNet(nin, nout, head)
    net.set_flat(glorot_init(rng, nin, nout, head))
    x = torch.randn(N, nin, device="cuda")
    gh = torch.randn(N * net.gh, device="cuda") * 1e-3
    partial = torch.zeros(net.partial_rows(N) * 4, dtype=torch.float64, device="cuda")
    if head == _lib.HEAD_LINEAR:
        net.rows(_lib.EPI_VFLOSS, x, N, inv_n_global=1.0 / N, target=torch.randn(N, device="cuda"), ghead=gh,
                 partial=partial)
    else:
        act = (torch.randint(0, nout, (N,), dtype=torch.int32, device="cuda") if head == _lib.HEAD_SOFTMAX
               else torch.randn(N, nout, device="cuda"))
        prob = net.forward(x, N).clone()
        net.rows(_lib.EPI_SURRGRAD, x, N, inv_n_global=1.0 / N, act=act, adv=torch.randn(N, device="cuda"),
                 oldprob=prob, ghead=gh, partial=partial)
    cache = net._cache(N)
    rows = int(net.lib.mrl_mlp_slab_rows(ctypes.byref(net.desc), N))
    slab = torch.zeros(rows * net.P, device="cuda")

    def launch():
        call("mrl_mlp_vjp", ctypes.byref(net.desc), ptr(net.image), ptr(x), None, 1.0, ptr(gh), N, ptr(slab),
             ptr(cache), None, stream())

    launch()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        launch()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    flop = 2.0 * (2 * 64 * 64 + 64 * nout * 2 + nin * 64) * N
    print(f"vjp16 nin={nin} nout={nout}: {ms:.3f} ms/launch "
          f"{flop / ms / 1e9:.1f} TFLOP/s = {flop / ms / 1e9 / 157.3:.3f} of fp32 MFMA", flush=True)
