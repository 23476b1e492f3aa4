"""Diagnostic driver: a few Humanoid-v2 collects (E envs x T steps, 3x512 policy) for
rocprofv3 counter passes over the wave-per-env step (hm_act_kernel)."""
import sys

import torch

sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent  # noqa: E402
from modular_rl_amd.envs import make  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dtype = sys.argv[3] if len(sys.argv) > 3 else "fp32"
env = make("Humanoid-v2")
cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=E, horizon=T, seed=0, use_graph=0, hid_sizes=[512, 512, 512],
           mlp_dtype=dtype)
ag = TrpoAgent(env.observation_space, env.action_space, cfg)
col = ag.make_collector(env, cfg)
for _ in range(2):
    col.collect()
torch.cuda.synchronize()
print("ok", E, T, flush=True)
