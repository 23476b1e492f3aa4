"""Diagnostic: per-phase shader-clock stamps of the Humanoid wave-per-env step
(hm_act_kernel, block 0, substep pass 1).  Prints the mean cycles of each phase over
steps 8..T-1, the kernel's cycles and the shader clock it ran at.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent  # noqa: E402
from modular_rl_amd.envs import make  # noqa: E402

NAMES = ["local", "world", "cinert+cdof", "cvel", "contact", "cacc", "subtree", "F+force", "M", "LDL", "solve"]
T = 64
env = make("Humanoid-v2")
for E in [int(x) for x in (sys.argv[1:] or ["1024"])]:
    cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=E, horizon=T, seed=0, use_graph=0,
               hid_sizes=[512, 512, 512])
    ag = TrpoAgent(env.observation_space, env.action_space, cfg)
    col = ag.make_collector(env, cfg)
    col.collect()
    st = torch.zeros(T * 16, dtype=torch.int64, device="cuda")
    col.stamps = st
    col.collect()
    torch.cuda.synchronize()
    raw = st.view(T, 16).cpu().numpy().astype(np.float64)[8:]
    d = np.diff(raw[:, :12], axis=1).mean(0)
    cyc = (raw[:, 14] - raw[:, 13]).mean()
    ns = ((raw[:, 15] - raw[:, 12]) * 10.0).mean()
    print("E", E, "kernel %.0f cycles %.1f us (%.2f GHz)" % (cyc, ns / 1e3, cyc / ns),
          "substep %.0f cycles" % (raw[:, 11] - raw[:, 0]).mean(), flush=True)
    print("  " + " ".join("%s %.0f" % (n, v) for n, v in zip(NAMES, d)), flush=True)
