"""A/B bit-identity of whole layered rollouts (Humanoid, fused head; fp32 and bf16) between
two builds of libmrl_hip.so: two collects of 256 envs x 32 steps each, every trajectory
buffer and the running filter saved.

    MRL_LIB_PATH=<a.so> python tools/rollout_ab.py run OUT_A.npz
    MRL_LIB_PATH=<b.so> python tools/rollout_ab.py run OUT_B.npz
    python tools/rollout_ab.py cmp OUT_A.npz OUT_B.npz     (exit 1 unless bit-identical)
"""
import sys

import numpy as np

sys.path.insert(0, ".")


def run(out):
    from modular_rl_amd import _lib
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.envs import make
    env = make("Humanoid-v2")
    res = {}
    for dt in ("fp32", "bf16"):
        cfg = dict(timestep_limit=env.spec.max_episode_steps, n_envs=256, horizon=32, seed=5, mlp_dtype=dt,
                   hid_sizes=[512, 512, 512], use_graph=0)
        agent = TrpoAgent(env.observation_space, env.action_space, cfg)
        col = agent.make_collector(env, cfg)
        for it in range(2):
            b = col.collect()
            for k in ("obs", "act", "prob", "rew", "flags", "ep_t"):
                res[f"{dt}_{it}_{k}"] = getattr(b, k).cpu().numpy()
            res[f"{dt}_{it}_filter"] = col.filter_state.cpu().numpy()
    np.savez(out, **res)
    print("saved", out, "via", _lib.LIB_PATH)


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        n = int((x[k].view(np.uint8) != y[k].view(np.uint8)).sum())
        bad += n
        if n:
            print(f"{k}: {n} bytes differ")
    print("BIT-IDENTICAL" if bad == 0 else "DIFFERENT", f"({len(x.files)} arrays)")
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
