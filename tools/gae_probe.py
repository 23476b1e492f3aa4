"""Time mrl_gae (scan + moments) alone at T x E (default the bench's 1024 x 4096);
MRL_LIB_PATH selects an ablation build (tools/build_ablate.sh)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd import _lib  # noqa: E402
from modular_rl_amd._lib import call, ptr, stream  # noqa: E402


def main(T=1024, E=4096, reps=50):
    g = torch.Generator(device='cuda').manual_seed(0)
    rew = torch.rand(T * E, device='cuda', generator=g)
    v = torch.randn(T * E, device='cuda', generator=g)
    flags = (torch.rand(T * E, device='cuda', generator=g) < 1 / 200).to(torch.uint8)
    adv = torch.empty_like(rew)
    ret = torch.empty_like(rew)
    mom = torch.zeros(3, dtype=torch.float64, device='cuda')
    ws = torch.zeros(int(_lib.load().mrl_gae_workspace_bytes(T, E)), dtype=torch.uint8, device='cuda')

    def run():
        call("mrl_gae", ptr(rew), ptr(v), ptr(flags), T, E, 0.995, 0.97, ptr(adv), ptr(ret), ptr(mom), ptr(ws), stream())

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = 17 * T * E / (ms * 1e-3) / 1e9
    lib = os.path.basename(os.environ.get("MRL_LIB_PATH", "default"))
    if os.environ.get("MRL_GAE_GENERAL") == "1":
        lib += ", general kernel"
    print(f"[{lib}] gae T={T} E={E}: {ms * 1e3:.1f} us/call back-to-back, {gbs:.0f} GB/s algorithmic, "
          f"mean adv {float(mom[0]) / (T * E):.5f}", flush=True)


if __name__ == "__main__":
    main()
    main(T=1024, E=1024)
