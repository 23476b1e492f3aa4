"""Probe: does the update write into the sync buffer, and does the replayed memset clear it?"""
import sys
import torch
sys.path.insert(0, ".")
from modular_rl_amd.agentzoo import TrpoAgent
from modular_rl_amd.envs import make


def head(col):
    torch.cuda.synchronize()
    h = col._sync.cpu().numpy()
    nz = [i for i in range(h.size) if h[i] != 0]
    return len(nz), nz[:4], [hex(int(x) & 0xffffffff) for x in h[nz[:4]]]


for graph in (1, 0, 1):
    env = make("Hopper-v2")
    cfg = dict(n_envs=64, horizon=64, timestep_limit=1000, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1,
               use_graph=graph, seed=3)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg)
    col = agent.make_collector(env, cfg)
    print("graph", graph, "sync %x..%x" % (col._sync.data_ptr(), col._sync.data_ptr() + 4 * col._sync.numel()))
    for i in range(3):
        b = col.collect()
        print("  after collect", head(col), flush=True)
        b.adv = torch.randn(b.n, device="cuda")
        ops = agent.updater.ops
        agent.updater.update(b)
        print("  after update", head(col), flush=True)
        for name in ("g", "fv", "b", "x", "ax", "r", "p", "p32", "fullstep", "cand", "cand_image", "tan_image", "state",
                     "flag", "step_out", "sums", "ghead", "partial"):
            t = getattr(ops, name, None)
            if t is not None and torch.is_tensor(t):
                lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
                if lo < col._sync.data_ptr() + 640 and hi > col._sync.data_ptr():
                    print("    OVERLAP", name, "%x..%x" % (lo, hi))
        for k, t in agent.policy.net.ws._bufs.items():
            lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()
            if lo < col._sync.data_ptr() + 640 and hi > col._sync.data_ptr():
                print("    OVERLAP ws", k, "%x..%x" % (lo, hi))
