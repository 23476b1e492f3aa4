"""Diagnostic: per-phase s_memrealtime stamps of the persistent rollout launch.

Block 0 stamps columns 0-7 of every step.  Phases: 0 step start | 1 every block's
step-t partials gathered (the tagged-granule hand-off; 7: the last granule arrived) and merged | 2 filtered obs |
3 forward | 4 sample + env step | 5 finish + raw obs in LDS | 6 partial published.
Prints the mean duration of each phase (ns) over steps 16..T-1.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent  # noqa: E402
from modular_rl_amd.envs import make  # noqa: E402

NAMES = ["gather+merge", "obs", "forward", "step", "finish", "publish"]
T = 256
args = [a for a in sys.argv[1:] if not a.startswith("--")]
dtype = "bf16" if "--bf16" in sys.argv else "fp32"
for env_id in args or ["Hopper-v2", "CartPole-v0"]:
    env = make(env_id)
    for E in [4096, 1024]:
        cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=E, horizon=T, seed=0, use_graph=0,
                   mlp_dtype=dtype)
        ag = TrpoAgent(env.observation_space, env.action_space, cfg)
        col = ag.make_collector(env, cfg)
        col.collect()
        # production kernel (no stamp code): mean of 3 collects
        torch.cuda.synchronize()
        p0 = torch.cuda.Event(enable_timing=True)
        p1 = torch.cuda.Event(enable_timing=True)
        p0.record()
        for _ in range(3):
            col.collect()
        p1.record()
        torch.cuda.synchronize()
        prod_ms = p0.elapsed_time(p1) / 3
        st = torch.zeros(T * 16, dtype=torch.int64, device="cuda")
        col.stamps = st
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        col.collect()
        e1.record()
        torch.cuda.synchronize()
        col.check()
        raw = st.view(T, 16).cpu().numpy().astype(np.float64) * 10.0  # ns
        s = raw[16:, :7]
        d = np.diff(s, axis=1).mean(0)
        tot = (raw[17:, 0] - raw[16:-1, 0]).mean()
        # column 7: the gather's last granule arrived (before the merge arithmetic)
        arr = (raw[16:, 7] - raw[16:, 0]).mean()
        mrg = (raw[16:, 8] - raw[16:, 7]).mean()  # column 8: block 0 wave 0's merge done (before the barrier)
        clk = st.view(T, 16).cpu().numpy()[:, 9].astype(np.float64)  # shader clock at step start
        ghz = (clk[-1] - clk[16]) / (raw[-1, 0] - raw[16, 0])
        print(env_id, E, "prod ms/collect %.3f (%.0f ns/step)" % (prod_ms, prod_ms * 1e6 / T),
              "stamped ms/collect %.3f" % e0.elapsed_time(e1), "step-to-step ns %.0f" % tot,
              " ".join("%s %.0f" % (n, v) for n, v in zip(NAMES, d)), "(arrival %.0f, merge %.0f) clock %.2f GHz" % (arr, mrg, ghz), flush=True)
