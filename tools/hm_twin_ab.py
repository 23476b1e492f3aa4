"""A/B bit-identity of the Humanoid step between two builds of libmrl_hip.so.

Runs the Humanoid step (mrl_rollout_act, z rows given, logstd 0, injected noise) for T
steps over E envs and saves every step's fp64 env state and raw observation + reward.

    MRL_LIB_PATH=<a.so> python tools/hm_twin_ab.py run OUT_A.npz
    MRL_LIB_PATH=<b.so> python tools/hm_twin_ab.py run OUT_B.npz
    python tools/hm_twin_ab.py cmp OUT_A.npz OUT_B.npz     (exit 1 unless bit-identical)
"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")


def run(out, E=256, T=64):
    import torch
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, ptr, stream
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.core import DiagGauss, StochPolicyMLP
    from modular_rl_amd.envs import make
    from modular_rl_amd.nets import LayeredMlpNet
    env = make("Humanoid-v2")
    A, O = env.act_dim, env.obs_dim
    net = LayeredMlpNet(O, A, _lib.HEAD_GAUSS, [32])
    col = Collector(env, StochPolicyMLP(net, DiagGauss(A)), E, T, 1000, filter=1, seed=31337, use_graph=False)
    rng = np.random.default_rng(7)
    col.set_noise(rng.standard_normal((T * E, A)))
    z = (0.4 * rng.standard_normal((T, E, A))).astype(np.float32)
    logstd = torch.zeros(A, dtype=torch.float32, device="cuda")
    d, bufs = ctypes.byref(col.desc), col._bufs()
    call("mrl_rollout_reset_rows", d, ctypes.byref(bufs), stream())
    states, raws = [], []
    for t in range(T):
        zt = torch.as_tensor(z[t]).cuda().contiguous()
        call("mrl_rollout_act", d, int(_lib.HEAD_GAUSS), A, ptr(zt), ptr(logstd), ctypes.byref(bufs), t, stream())
        states.append(col.env_state[:64 * E].clone())  # the state rows (not the kinematics cache)
        raws.append(col.raw_obs.clone())
    torch.cuda.synchronize()
    np.savez(out, state=torch.stack(states).cpu().numpy(), raw=torch.stack(raws).cpu().numpy(),
             flags=col.flags.cpu().numpy())
    print("saved", out, "via", _lib.LIB_PATH)


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        n = int((x[k].view(np.uint8) != y[k].view(np.uint8)).sum()) if x[k].dtype != np.float64 else \
            int((x[k].view(np.uint64) != y[k].view(np.uint64)).sum())
        print(f"{k}: {x[k].size} words, {n} differ")
        bad += n
    print("BIT-IDENTICAL" if bad == 0 else "DIFFERENT")
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
