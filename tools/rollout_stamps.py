"""Diagnostic: per-phase s_memrealtime stamps of one rollout_step launch (block 0)."""
import sys, torch, numpy as np
sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent
from modular_rl_amd.envs import make
for env_id in ["Hopper-v2", "CartPole-v0"]:
    env = make(env_id)
    for E in [4096, 128]:
        cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=E, horizon=256, seed=0, use_graph=0)
        ag = TrpoAgent(env.observation_space, env.action_space, cfg)
        col = ag.make_collector(env, cfg)
        col.collect()
        st = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
        col.stamps = st
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); col.collect(); e1.record(); torch.cuda.synchronize()
        s = st.view(256, 8).cpu().numpy().astype(np.float64) * 10.0  # ns
        d = np.diff(s, axis=1)[16:]   # skip first steps
        tot = (s[17:, 0] - s[16:-1, 0]).mean()
        print(env_id, E, "ms/collect %.2f" % e0.elapsed_time(e1), "step-to-step ns %.0f" % tot,
              "phases ns:", " ".join("%.0f" % v for v in d.mean(0)))
