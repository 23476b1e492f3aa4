"""Diagnostic: per-phase s_memrealtime stamps of one rollout_step launch (block 0).

Phases (rollout.hip STAMP ids in time order): 0 start | 1 loads issued | 2 filter merge |
3 filtered obs | 9 forward layer 0 | 10 layer 1 | 4 head | 5 sample+env step |
6 finish+obs+sync | 7 publish partial.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent  # noqa: E402
from modular_rl_amd.envs import make  # noqa: E402

ORDER = [0, 1, 2, 3, 9, 10, 4, 5, 6, 7]
NAMES = ["issue", "filter", "obs", "fwd-l0", "fwd-l1", "head", "step", "finish", "publish"]
T = 256
for env_id in ["Hopper-v2", "CartPole-v0"]:
    env = make(env_id)
    for E in [4096, 128]:
        cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=E, horizon=T, seed=0, use_graph=0)
        ag = TrpoAgent(env.observation_space, env.action_space, cfg)
        col = ag.make_collector(env, cfg)
        col.collect()
        st = torch.zeros(T * 16, dtype=torch.int64, device="cuda")
        col.stamps = st
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        col.collect()
        e1.record()
        torch.cuda.synchronize()
        raw = st.view(T, 16).cpu().numpy().astype(np.float64)
        ghz = np.median((raw[16:, 15] - raw[16:, 14]) / ((raw[16:, 7] - raw[16:, 0]) * 10.0))
        s = raw[:, ORDER] * 10.0  # ns
        d = np.diff(s, axis=1)[16:]  # skip the first steps
        tot = (s[17:, 0] - s[16:-1, 0]).mean()
        print(env_id, E, "ms/collect %.2f" % e0.elapsed_time(e1), "step-to-step ns %.0f" % tot, "clock %.2f GHz" % ghz,
              " ".join("%s %.0f" % (n, v) for n, v in zip(NAMES, d.mean(0))), flush=True)
