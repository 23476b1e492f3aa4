"""Checkpoint / resume and run diagnostics.

The reference snapshots the whole agent as a pickle inside an HDF5 file
(`run_pg.py:141-142`: ``hdf['/agent_snapshots/%0.4i'] = cPickle.dumps(agent)``) and
logs per-iteration scalars into ``hdf['diagnostics']`` (`misc_utils.py:111-132`);
``load_snapshot`` is declared but never read (`misc_utils.py:102`).  Here the agent
state is a flat set of arrays -- nothing executable is ever stored or loaded:

  policy/theta, vf/theta            fp32 flat parameters (Keras trainable_weights order)
  filter/state                      ZFilter running stats (n, n_rew, mean[D], M2[D], fp64)
  rng/iteration, rng/episodes       device Philox step base and per-env episode counters,
                                    so a resumed run draws exactly the noise the
                                    uninterrupted run would have drawn
  rng/np_mt19937, rng/np_pos_gauss  numpy's global MT19937 state (PpoSgd's minibatch
                                    permutations)
  updater/*                         the policy updater's own state (PPO: kl_coeff, the
                                    Adam moments and step count) -- the reference keeps
                                    it by pickling the whole agent
  meta (JSON)                       cfg, env id, iteration counter

In the pipelined loop (core.IterationRunner) the callback for iteration k fires
after iteration k+1 has already been issued; the runner therefore captures the state
at the end of iteration k on the device (``agent._snapshot_capture``) and snapshots
taken in that callback read the capture, not the live tensors.  The capture is
dropped when the callback returns (``run_policy_gradient_algorithm``), so a snapshot
taken later -- after a manual ``set_from_flat`` or another update -- reads the live
state.

Snapshots are ``.npz`` files (``numpy.load(allow_pickle=False)`` reads them); the run
log is HDF5 with the reference's layout when ``h5py`` is importable, else an ``.npz``
with the same keys (``params`` as JSON, ``diagnostics/<stat>`` arrays, ``cmd``).
"""
import json
import os
import sys
from collections import defaultdict

import numpy as np
import torch

# 2: updater/* (PPO Adam moments, step count, kl_coeff) and rng/np_* arrays were added;
# a version-1 snapshot has neither, so it loads only into agents whose updater keeps no
# state of its own (TRPO)
SNAPSHOT_VERSION = 2


def _jsonable(cfg):
    out = {}
    for k, v in (cfg or {}).items():
        try:
            json.dumps(v)
            out[k] = v
        except TypeError:
            out[k] = repr(v)
    return out


def _host(v):
    return v.detach().cpu().numpy().copy() if torch.is_tensor(v) else np.array(v, copy=True)


def capture_state(agent, with_vf=True, host=True, theta=True):
    """Device-side copies (stream-ordered, no host sync) of everything agent_state
    saves; the pipelined runner takes one at the end of each iteration.  host=False:
    only the state the next rollout advances (taken before that rollout is issued; the
    rest, capture_host_state, after it); theta=False: without the policy parameters
    (the runner clones them after issuing that rollout, which only reads them)."""
    cap = {"policy/theta": agent.policy.net.theta.detach().clone()} if theta else {}
    if with_vf:
        cap["vf/theta"] = agent.baseline.net.theta.detach().clone()
    col = agent._filter_owner()
    if col is not None:
        cap["filter/state"] = col.filter_state[:col.FS].detach().clone()
        cap["rng/iteration"] = col.iteration.detach().clone()
        cap["rng/episodes"] = col.env_int[col.E:].detach().clone()
    if host:
        cap.update(capture_host_state(agent))
    return cap


def capture_host_state(agent):
    """The part of capture_state no rollout touches: numpy's RNG and the updater's
    own state arrays."""
    cap = {}
    # numpy's global MT19937 (PpoSgd draws its minibatch permutations from it, as the
    # reference does): saved as arrays so a resumed run permutes identically
    name, keys, pos, has_gauss, gauss = np.random.get_state()
    cap["rng/np_mt19937"] = np.array(keys, dtype=np.uint32)
    cap["rng/np_pos_gauss"] = np.array([pos, has_gauss, gauss], dtype=np.float64)
    upd = getattr(agent, "updater", None)
    if upd is not None and hasattr(upd, "state_arrays"):
        for k, v in upd.state_arrays().items():
            cap["updater/" + k] = v.detach().clone() if torch.is_tensor(v) else np.array(v, copy=True)
    return cap


def agent_state(agent, counter=0, env_id=None):
    """Arrays (+ JSON meta) that restore ``agent`` to this point of training: the
    pipelined runner's capture of the iteration last reported, else the live state."""
    cap = getattr(agent, "_snapshot_capture", None) or capture_state(agent)
    st = {k: _host(v) for k, v in cap.items()}
    meta = dict(version=SNAPSHOT_VERSION, counter=int(counter), env_id=env_id, cfg=_jsonable(agent.cfg))
    return st, meta


def save_snapshot(path, agent, counter=0, env_id=None):
    st, meta = agent_state(agent, counter, env_id)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    arrays = {k.replace("/", "__"): v for k, v in st.items()}
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)
    return path


def load_snapshot(path, agent):
    """Restore parameters now; filter / RNG state go to the agent's collector (applied
    immediately if it exists, else when ``make_collector`` creates it)."""
    with np.load(path, allow_pickle=False) as z:
        st = {k.replace("__", "/"): z[k] for k in z.files if k != "meta"}
        meta = json.loads(bytes(z["meta"]).decode())
    version = meta.get("version")
    upd = getattr(agent, "updater", None)
    if version == 1:
        if upd is not None and hasattr(upd, "state_arrays"):
            raise ValueError(f"{path}: version-1 snapshot holds no updater state (Adam moments, kl_coeff), "
                             f"which this agent's {type(upd).__name__} needs to resume exactly")
    elif version != SNAPSHOT_VERSION:
        raise ValueError(f"{path}: snapshot version {version} != {SNAPSHOT_VERSION}")
    pol, vf = agent.policy.net, agent.baseline.net
    if st["policy/theta"].shape != (pol.P,) or st["vf/theta"].shape != (vf.P,):
        raise ValueError(f"{path}: parameter shapes do not match this agent's nets")
    pol.set_flat(st["policy/theta"])
    vf.set_flat(st["vf/theta"])
    upd_state = {k[len("updater/"):]: v for k, v in st.items() if k.startswith("updater/")}
    if upd_state:
        if upd is None or not hasattr(upd, "load_state_arrays"):
            raise ValueError(f"{path}: snapshot holds updater state this agent's updater cannot take")
        upd.load_state_arrays(upd_state)
    if "rng/np_mt19937" in st:
        pos, has_gauss, gauss = st["rng/np_pos_gauss"]
        np.random.set_state(("MT19937", st["rng/np_mt19937"].astype(np.uint32), int(pos), int(has_gauss), float(gauss)))
    agent._snapshot_capture = None
    agent._pending_state = {k: v for k, v in st.items() if k.startswith(("filter/", "rng/"))
                            and not k.startswith("rng/np_")}
    col = agent._filter_owner()
    if col is not None:
        apply_collector_state(col, agent._pending_state)
        agent._pending_state = None
    return meta


def apply_collector_state(col, st):
    if not st:
        return
    if "filter/state" in st:
        fs = torch.as_tensor(st["filter/state"], dtype=torch.float64)
        if fs.numel() != col.FS:
            raise ValueError("snapshot filter state does not match the env")
        col.filter_state[:col.FS].copy_(fs.to(col.filter_state.device))
    if "rng/iteration" in st:
        col.iteration.copy_(torch.as_tensor(st["rng/iteration"], dtype=torch.int64).to(col.iteration.device))
    if "rng/episodes" in st:
        ep = torch.as_tensor(st["rng/episodes"], dtype=torch.int32)
        if ep.numel() != col.E:
            raise ValueError(f"snapshot has episode counters for {ep.numel()} envs, this collector steps {col.E}")
        col.env_int[col.E:].copy_(ep.to(col.env_int.device))


class RunLog:
    """The reference's ``prepare_h5_file`` (`misc_utils.py:111-132`): params, per-iteration
    scalar diagnostics, agent snapshots, env id and the command line."""

    def __init__(self, fname, args):
        self.fname = fname
        self.params = _jsonable(vars(args) if not isinstance(args, dict) else args)
        self.diagnostics = defaultdict(list)
        self.snapshots = {}
        self.extra = {"cmd": " ".join(sys.argv)}
        try:
            import h5py  # noqa: F401
            self.h5 = True
        except ImportError:
            self.h5 = False

    def record(self, stats):
        for k, v in stats.items():
            a = np.asarray(v)
            if a.ndim == 0:
                self.diagnostics[k].append(float(a))
            else:
                self.diagnostics[k].extend(a.ravel().tolist())

    def snapshot(self, counter, agent, env_id=None):
        st, meta = agent_state(agent, counter, env_id)
        self.snapshots["%0.4i" % counter] = (st, meta)

    def save(self):
        d = os.path.dirname(os.path.abspath(self.fname))
        os.makedirs(d, exist_ok=True)
        if self.h5:
            import h5py
            with h5py.File(self.fname, "w") as f:
                g = f.create_group("params")
                for k, v in self.params.items():
                    try:
                        g[k] = v
                    except (TypeError, ValueError):
                        g[k] = json.dumps(v)
                dg = f.create_group("diagnostics")
                for k, v in self.diagnostics.items():
                    dg[k] = np.asarray(v)
                for name, (st, meta) in self.snapshots.items():
                    sg = f.create_group("agent_snapshots/" + name)
                    for k, v in st.items():
                        sg[k] = v
                    sg.attrs["meta"] = json.dumps(meta)
                for k, v in self.extra.items():
                    f[k] = v
            return self.fname
        arrays = {"params": np.frombuffer(json.dumps(self.params).encode(), dtype=np.uint8)}
        for k, v in self.diagnostics.items():
            arrays["diagnostics__" + k] = np.asarray(v, dtype=np.float64)
        for name, (st, meta) in self.snapshots.items():
            for k, v in st.items():
                arrays[f"agent_snapshots__{name}__{k.replace('/', '__')}"] = v
            arrays[f"agent_snapshots__{name}__meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        for k, v in self.extra.items():
            arrays[k] = np.frombuffer(str(v).encode(), dtype=np.uint8)
        out = self.fname if self.fname.endswith(".npz") else os.path.splitext(self.fname)[0] + ".npz"
        np.savez(out, **arrays)
        return out
