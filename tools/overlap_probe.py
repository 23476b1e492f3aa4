"""Can the VF fit of iteration k overlap the rollout of iteration k+1?  Times, at the
bench config (Hopper 4096 x 1024), the rollout graph replay and the VF L-BFGS fit
alone on the default stream, alone on CU-masked streams, and both at once."""
import sys
import time

import torch

sys.path.insert(0, '.')
from modular_rl_amd.agentzoo import TrpoAgent  # noqa: E402
from modular_rl_amd.core import compute_advantage_batch  # noqa: E402
from modular_rl_amd.envs import make  # noqa: E402
from modular_rl_amd import streams  # noqa: E402


def wall(fn, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    env = make("Hopper-v2")
    cfg = dict(timestep_limit=env.spec.max_episode_steps, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1,
               n_envs=4096, horizon=1024, filter=1, seed=0, hid_sizes=[64, 64], activation="tanh", use_graph=1)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    col = agent.make_collector(env, cfg)
    batch = col.collect()
    compute_advantage_batch(agent.baseline, batch, 0.995, 0.97)
    agent.baseline.fit_batch(batch)
    agent.updater.update(batch)
    torch.cuda.synchronize()
    ncu = streams.cu_count()
    print(f"CUs: {ncu}", flush=True)
    fit = lambda: agent.baseline.fit_batch(batch)  # noqa: E731
    roll = lambda: col.collect()  # noqa: E731
    print(f"default stream: rollout {wall(roll):.2f} ms, vf fit {wall(fit):.2f} ms", flush=True)
    layouts = {
        "lo64": list(range(64)),
        "stride4": list(range(0, ncu, 4)),
        "lo96": list(range(96)),
        "stride8x2": [c for c in range(ncu) if (c % 8) < 2],
    }
    for name, rc in layouts.items():
        vc = [c for c in range(ncu) if c not in set(rc)]
        R, V = streams.masked_stream(rc), streams.masked_stream(vc)
        got = streams.stream_cus(R)
        def roll_r():
            with torch.cuda.stream(R):
                col.collect()
        def fit_v():
            with torch.cuda.stream(V):
                agent.baseline.fit_batch(batch)
        def both():
            with torch.cuda.stream(R):
                col.collect()
            with torch.cuda.stream(V):
                agent.baseline.fit_batch(batch)
        tr, tv, tb = wall(roll_r), wall(fit_v), wall(both)
        print(f"{name}: R={len(rc)} CUs (mask readback {len(got)}), V={len(vc)}: rollout {tr:.2f} ms, "
              f"vf fit {tv:.2f} ms, both {tb:.2f} ms (sum {tr + tv:.2f})", flush=True)


if __name__ == "__main__":
    main()
