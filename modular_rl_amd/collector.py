"""Lock-step batched rollout collector (replaces get_paths / do_rollouts_serial /
rollout, `core.py:174-221`).

E envs per rank advance together for ``horizon`` steps per iteration.  With the
fused 64-wide policy each step is ONE HIP launch (filter merge -> normalise ->
policy MLP on MFMA -> sample -> env step -> Welford partials).  With a layered
policy (wide nets, Humanoid's 376-d obs) a step is mrl_rollout_obs -> the policy's
GEMM forward over the E rows -> mrl_rollout_act.  The T launches (plus reset/finish) can be captured
once into a hipGraph and replayed every iteration (``use_graph``): the policy
weights are read through persistent buffers (theta / the rollout image repacked at
the head of every replay) and the RNG step base
from a device iteration counter, so replays need no re-capture.

Semantics vs the reference: every env is reset at the start of
an iteration (core.py:186); observations are stored filtered, rewards raw; an
episode ends at env ``done`` (gym TimeLimit included => terminated, bootstrap 0) or
at the ``timestep_limit`` / horizon cut (not terminated, bootstrap b[-1]).  The
ZFilter pushes all E observations of a step as one Chan merge (E = 1 reduces
exactly to RunningStat.push); across ranks the running stats are merged once per
iteration (rank order), so ranks normalise with identical statistics at every
iteration start.
"""
import ctypes
import gc
import os

import numpy as np
import torch

from . import _lib, timing
from ._lib import call, ptr, stream
from .dist import Comm


def _chan_delta(s0, s1, D):
    """A rank's pushes of one iteration as (n, mean, M2) per column: Chan's merge
    s1 = s0 (+) delta inverted."""
    delta = np.zeros(len(s0))
    for which, cols in ((0, range(D - 1)), (1, [D - 1])):
        n0, n1 = s0[which], s1[which]
        nd = n1 - n0
        delta[which] = nd
        if nd <= 0:
            continue
        for k in cols:
            M0, M1, S0, S1 = s0[2 + k], s1[2 + k], s0[2 + D + k], s1[2 + D + k]
            md = (n1 * M1 - n0 * M0) / nd
            delta[2 + k] = md
            delta[2 + D + k] = S1 - S0 - (md - M0) ** 2 * n0 * nd / n1
    return delta


def merge_filter_deltas(s0, s1, comm):
    """Per-iteration cross-rank merge of the running stats.  Every rank started the
    iteration from the same state s0 = [n_obs, n_rew, M[D], S[D]] and ended at its
    local s1 = s0 (+) its own pushes.  All ranks' end states are gathered; rank 0's is
    the base and the pushes of ranks 1, 2, .. (each recovered by inverting Chan's
    formula against s0) are merged into it in rank order, so all ranks leave with the
    identical global statistics -- and one rank (a forced communicator at world size 1)
    leaves with its own s1 exactly."""
    FS = len(s0)
    D = (FS - 2) // 2
    dev = "cuda" if comm.enabled and torch.distributed.get_backend() == "nccl" else "cpu"
    s1_t = torch.as_tensor(np.asarray(s1, dtype=np.float64)).to(dev)
    all_s1 = torch.stack(comm.allgather(s1_t)).cpu().numpy()  # one copy for all ranks
    s0 = np.asarray(s0, dtype=np.float64)
    out = all_s1[0].copy()
    for s1r in all_s1[1:]:
        d = _chan_delta(s0, s1r, D)
        for which, cols in ((0, range(D - 1)), (1, [D - 1])):
            nb = d[which]
            if nb <= 0:
                continue
            n = out[which] + nb
            for k in cols:
                M, S = out[2 + k], out[2 + D + k]
                mb, m2b = d[2 + k], d[2 + D + k]
                dl = mb - M
                newM = M + (dl * nb) / n
                out[2 + D + k] = S + m2b + dl * (mb - newM) * nb
                out[2 + k] = newM
            out[which] = n
    return out


class Batch:
    """Device-resident batch of N = T*E time-major rows (row n = t*E + e)."""

    def __init__(self, n, obs, act, prob, rew=None, flags=None, ep_t=None, T=None, E=None):
        self.n = int(n)
        self.obs, self.act, self.prob, self.rew, self.flags, self.ep_t = obs, act, prob, rew, flags, ep_t
        self.T, self.E = T, E
        self.adv = self.ret = self.vpred = None
        self.vf_x = None  # (VF features, NnVf feature generation) set by NnVf.predict_batch
        self.episode = None
        self.n_global = None  # rows over all ranks when the producer knows it (Collector)
        self.rows_owner = self.rows_gen = None  # the collector whose buffers hold the rows

    def rows_valid(self):
        """False once the producing collector has launched another rollout into the same
        buffers (the pipelined loop issues the next rollout before this batch's VF fit)."""
        return self.rows_owner is None or self.rows_owner.rows_gen == self.rows_gen

    def check_abort(self, comm):
        """Raise before an update touches theta if this batch's persistent rollout gave up
        (any rank).  TrpoUpdater reads the status inside its first readback instead."""
        abort = getattr(self, "abort", None)
        if abort is None:
            return
        a = abort.double().reshape(1).clone()
        comm.allreduce_(a)
        if float(a.item()) != 0:
            raise _lib.MrlError("policy update on an aborted rollout: " + getattr(self, "abort_msg", ""))

    @staticmethod
    def from_paths(paths, stochpol, device, need_policy=True):
        """Concatenate per-path dicts (core.py:205-207 schema) into a device batch
        (one env, paths laid end to end: T = total rows, E = 1)."""
        cat = np.concatenate
        dev = torch.device(device)
        obs = torch.as_tensor(cat([np.asarray(p["observation"], dtype=np.float32) for p in paths])).to(dev)
        n = obs.shape[0]
        act = prob = None
        if need_policy:
            a = cat([np.asarray(p["action"]) for p in paths])
            act = torch.as_tensor(a.astype(np.int32) if stochpol.discrete else a.astype(np.float32)).to(dev)
            prob = torch.as_tensor(cat([np.asarray(p["prob"], dtype=np.float32) for p in paths])).to(dev)
        ep_t = torch.as_tensor(cat([np.arange(len(p["observation"]), dtype=np.int32) for p in paths])).to(dev)
        flags = np.zeros(n, dtype=np.uint8)
        ends = np.cumsum([len(p["observation"]) for p in paths]) - 1
        for e_, p in zip(ends, paths):
            flags[e_] = 1 | (2 if p.get("terminated", False) else 0)
        rew = None
        if "reward" in paths[0]:
            rew = torch.as_tensor(cat([np.asarray(p["reward"], dtype=np.float32) for p in paths])).to(dev)
        b = Batch(n, obs, act, prob, rew, torch.as_tensor(flags).to(dev), ep_t, T=n, E=1)
        if "advantage" in paths[0]:
            b.adv = torch.as_tensor(cat([np.asarray(p["advantage"], dtype=np.float32) for p in paths])).to(dev)
        return b

    def to_paths(self):
        """Split back into reference-style path dicts (host numpy), env by env."""
        T, E = self.T, self.E
        obs = self.obs.view(T, E, -1).cpu().numpy()
        act = self.act.view(T, E, *self.act.shape[1:]).cpu().numpy()
        prob = self.prob.view(T, E, -1).cpu().numpy()
        rew = self.rew.view(T, E).cpu().numpy().astype(np.float64)
        flags = self.flags.view(T, E).cpu().numpy()
        paths = []
        for e in range(E):
            start = 0
            for t in range(T):
                if flags[t, e] & 1:
                    sl = slice(start, t + 1)
                    paths.append(dict(observation=obs[sl, e], action=act[sl, e], prob=prob[sl, e],
                                      reward=rew[sl, e], terminated=bool(flags[t, e] & 2)))
                    start = t + 1
        return paths


class Collector:
    def __init__(self, env, policy, n_envs, horizon, timestep_limit, filter=1, seed=0, comm=None, device="cuda",
                 use_graph=False):
        lib = _lib.load(require_gpu=True)
        self.env, self.policy = env, policy
        self.comm = comm if comm is not None else Comm()
        self.E, self.T = int(n_envs), int(horizon)
        self.N = self.E * self.T
        # rows over all ranks, once per collector: the updates and the VF fit scale by it
        # without a host-synchronising all-reduce of a constant per call (core.py:123-124)
        self.N_global = self.comm.allreduce_int(self.N) if self.comm.enabled else self.N
        self.rows_gen = 0  # bumped by every launch: the batch rows it overwrites
        self.dev = torch.device(device)
        self.desc = _lib.RolloutDesc(env.kind, self.E, self.T, int(timestep_limit), int(filter),
                                     self.comm.rank * self.E, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                     _lib.COMPUTE[getattr(policy.net, "dtype", "fp32")], 0)
        ns = lib.mrl_env_state_doubles(env.kind)
        self.FS = int(lib.mrl_filter_doubles(env.kind))
        self.RS = int(lib.mrl_record_doubles(env.kind))
        self.NB = int(lib.mrl_rollout_blocks(self.E))
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.env_state = torch.zeros(ns * self.E, **f64)
        self.env_int = torch.zeros(2 * self.E, dtype=torch.int32, device=self.dev)
        self.filter_state = torch.zeros(2 * self.FS, **f64)
        self.records = torch.zeros(2 * self.NB * self.RS, **f64)
        self.iteration = torch.zeros(1, dtype=torch.int64, device=self.dev)
        O, A = env.obs_dim, env.act_dim
        self.obs = torch.zeros(self.N, O, dtype=torch.float32, device=self.dev)
        if env.discrete:
            self.act = torch.zeros(self.N, dtype=torch.int32, device=self.dev)
            self.prob = torch.zeros(self.N, A, dtype=torch.float32, device=self.dev)
        else:
            self.act = torch.zeros(self.N, A, dtype=torch.float32, device=self.dev)
            self.prob = torch.zeros(self.N, 2 * A, dtype=torch.float32, device=self.dev)
        self.rew = torch.zeros(self.N, dtype=torch.float32, device=self.dev)
        self.flags = torch.zeros(self.N, dtype=torch.uint8, device=self.dev)
        self.ep_t = torch.zeros(self.N, dtype=torch.int32, device=self.dev)
        self.noise = None  # injected noise rows (parity mode); None: Philox rows drawn per iteration
        self._noise_rows = torch.zeros(int(lib.mrl_rollout_noise_doubles(ctypes.byref(self.desc))), **f64)
        self.stamps = None  # diagnostic [T, 16] int64 phase stamps (see rollout.hip); None in production
        net = policy.net
        self.layered = bool(getattr(net, "layered", False))
        # Humanoid steps one env per wave (humanoid.h): its chain wants one wave per SIMD
        self.wave_per_env = env.kind == _lib.ENV_HUMANOID
        if env.kind == _lib.ENV_HUMANOID and not self.layered:
            raise _lib.MrlError("Humanoid-v2 needs a layered policy net (its 376-d obs exceeds the fused kernel)")
        self.raw_obs = None
        self.hidden_b16 = False
        if self.layered:
            # persistent per-step buffers (their addresses are baked into the captured graph)
            self.raw_obs = torch.zeros((O + 1) * self.E, **f64)
            self._zrows = torch.zeros(self.E * A, dtype=torch.float32, device=self.dev)
            w = max(net.hid_sizes)
            self._fwd_bufs = [torch.zeros(self.E * w, dtype=torch.float32, device=self.dev) for _ in range(2)]
            # bf16 tape mode, Humanoid: the hidden layers on the bf16 GEMMs (bf16 rows)
            self.hidden_b16 = self.wave_per_env and bool(getattr(net, "tape_bf16", False))
            if self.hidden_b16:
                i16 = dict(dtype=torch.int16, device=self.dev)
                self._fwd_b16 = [torch.zeros(self.E * w, **i16) for _ in range(2)]
                self._xb16 = torch.zeros(self.E * ((O + 7) // 8 * 8), **i16)
        else:
            # fused step kernel: its own policy image, repacked from theta at every collect
            n = int(lib.mrl_rollout_image_floats(ctypes.byref(net.desc)))
            self._rimage = torch.zeros(n, dtype=torch.float32, device=self.dev)
            nsync = int(lib.mrl_rollout_sync_bytes(ctypes.byref(self.desc)))
            self._sync = torch.zeros((nsync + 3) // 4, dtype=torch.int32, device=self.dev)
        # the whole horizon as one persistent launch (MRL_ROLLOUT_PERSISTENT=0: step launches)
        self.persistent = os.environ.get("MRL_ROLLOUT_PERSISTENT", "1") != "0"
        self.use_graph = use_graph
        self.graph = None
        self._ep_ws = torch.zeros(int(lib.mrl_episode_stats_workspace_bytes(self.E)) // 8 + 1, **f64)
        self._ep_out = torch.zeros(8, **f64)
        # sticky abort status of the persistent launch: sync[32] of every launch is OR-ed
        # in on the device (the next launch's memset clears sync); read back with the
        # episode stats each iteration, which raise MrlError when it is set
        self.status = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.force_persistent = False  # debug: skip the residency check (tests of the abort path)
        self._graph_cus = None

    def _bufs(self):
        return _lib.RolloutBufs(ptr(self.env_state), ptr(self.env_int), ptr(self.filter_state), ptr(self.records),
                                ptr(self.iteration), ptr(self.obs), ptr(self.act), ptr(self.prob), ptr(self.rew),
                                ptr(self.flags), ptr(self.ep_t),
                                ptr(self.noise if self.noise is not None else self._noise_rows), ptr(self.stamps),
                                ptr(self.raw_obs), ptr(self._xb16 if self.hidden_b16 else None))

    def fill_noise(self):
        """This iteration's sampling noise, one parallel draw over every row (no-op when
        noise is injected).  Issued outside the captured step graph so the pipelined
        loop can run it on all CUs while the step chain runs on the rollout's CU set."""
        if self.noise is None:
            call("mrl_rollout_noise", ctypes.byref(self.desc), ctypes.byref(self._bufs()), ptr(self._noise_rows),
                 stream())

    def _launch_all(self):
        bufs = self._bufs()
        net = self.policy.net
        if self.layered:
            return self._launch_all_layered(bufs, net)
        call("mrl_rollout_pack", ctypes.byref(self.desc), ctypes.byref(net.desc), ptr(net.theta), ptr(self._rimage),
             stream())
        # reset + T steps: one persistent cooperative launch (or T step launches when
        # persistent is off / the stream has too few CUs; identical results)
        call("mrl_rollout_run", ctypes.byref(self.desc), ctypes.byref(net.desc), ptr(net.theta), ptr(self._rimage),
             ctypes.byref(bufs), ptr(self._sync), int(self.persistent), stream())
        if self.persistent:
            torch.maximum(self.status, self._sync[32:33], out=self.status)
        call("mrl_rollout_finish", ctypes.byref(self.desc), ctypes.byref(bufs), stream())

    def _launch_all_layered(self, bufs, net):
        E, O = self.E, self.env.obs_dim
        d = ctypes.byref(self.desc)
        logstd = net._addr(net.theta, net.tls) if net.head == _lib.HEAD_GAUSS else None
        call("mrl_rollout_reset_rows", d, ctypes.byref(bufs), stream())
        L = len(net.dims) - 1
        wt = net.rollout_images() if self.hidden_b16 else None
        for t in range(self.T):
            call("mrl_rollout_obs", d, ctypes.byref(bufs), int(t), stream())
            x = self.obs[t * E:(t + 1) * E]
            if self.hidden_b16:
                # mrl_rollout_obs wrote the step's rows into _xb16 as bf16 too (obs_bf16)
                hid = net.forward_hidden_rows_b16(x, E, wt, self._fwd_b16, self._xb16, cast=False)
                call("mrl_rollout_act_head_bf16", d, int(net.head), int(net.n_out), ptr(hid), int(net.dims[L - 1]),
                     net._addr(net.theta, net.w_off[L - 1]), net._addr(net.theta, net.b_off[L - 1]), logstd,
                     ctypes.byref(bufs), int(t), stream())
            elif self.wave_per_env:
                # Humanoid: the head (1024 x 512 x 17, a thin GEMM) runs inside the step
                hid = net.forward_hidden_rows(x, E, self._fwd_bufs)
                call("mrl_rollout_act_head", d, int(net.head), int(net.n_out), ptr(hid), int(net.dims[L - 1]),
                     net._addr(net.theta, net.w_off[L - 1]), net._addr(net.theta, net.b_off[L - 1]), logstd,
                     ctypes.byref(bufs), int(t), stream())
            else:
                net.forward_rows(x, E, self._zrows, self._fwd_bufs)
                call("mrl_rollout_act", d, int(net.head), int(net.n_out), ptr(self._zrows), logstd,
                     ctypes.byref(bufs), int(t), stream())
        call("mrl_rollout_finish", d, ctypes.byref(bufs), stream())

    def set_noise(self, noise):
        """Inject sampling noise (float64 u[N] or z[N, d]) instead of Philox (parity mode)."""
        self.noise = None if noise is None else torch.as_tensor(noise, dtype=torch.float64).to(self.dev).contiguous()
        self.graph = None

    def collect(self):
        self.launch()
        return self.finish()

    def launch(self, fill_noise=True):
        """Issue one iteration's rollout on the current stream (asynchronous);
        ``fill_noise=False``: the caller already issued fill_noise() in stream order."""
        if fill_noise:
            self.fill_noise()
        self.rows_gen += 1
        self._fs_start = self.filter_state[:self.FS].clone() if self.comm.enabled else None
        # the persistent launch's residency check counts the CUs of the stream it runs on:
        # the stream of this call (a captured graph replays here, not on its capture stream)
        from . import streams
        self.desc.launch_cus = -1 if self.force_persistent else streams.launch_cus()
        # the persistent fused rollout is a handful of launches: replaying them as a graph
        # only adds the graph's launch latency (MRL_ROLLOUT_GRAPH=1 keeps it); the step-
        # launch rollouts (layered, or persistent off) replay their T x k launches
        graph = self.use_graph and self.noise is None and (
            self.layered or not self.persistent or os.environ.get("MRL_ROLLOUT_GRAPH", "auto") == "1")
        if graph:
            if self.graph is not None and self._graph_cus != self.desc.launch_cus:
                self.graph = None  # captured for another CU set
            if self.graph is None:
                self._graph_cus = self.desc.launch_cus
                # captured launches are recorded, not executed: state is untouched by the
                # capture.  No garbage collection inside the capture: collecting a dead
                # object that owns HIP state (an earlier collector's graph) while the
                # stream captures fails in its destructor and aborts the process.
                gc.collect()
                self.graph = torch.cuda.CUDAGraph()
                gc_was = gc.isenabled()
                gc.disable()
                try:
                    with torch.cuda.graph(self.graph):
                        self._launch_all()
                finally:
                    if gc_was:
                        gc.enable()
            timing.start("rollout_steps")
            self.graph.replay()
            timing.stop("rollout_steps")
        else:
            timing.start("rollout_steps")
            self._launch_all()
            timing.stop("rollout_steps")

    ABORT_MSG = ("persistent rollout: blocks never all arrived (grid not resident), the trajectories are "
                 "incomplete; run with MRL_ROLLOUT_PERSISTENT=0")

    def check(self):
        """Raise if a persistent rollout launch gave up waiting for its blocks (the grid
        was not resident at once); synchronises on the rollout."""
        if int(self.status.item()) != 0:
            raise _lib.MrlError(self.ABORT_MSG)

    def finish(self):
        """Cross-rank filter merge (waits for the rollout) and the iteration's Batch.  The
        batch carries the device abort status, which the policy update reads back with its
        step scalars before it touches theta."""
        if self.comm.enabled:
            # the merge synchronises on the rollout anyway: an aborted rollout must not
            # merge its partial filter deltas into every rank's filter
            self.check()
            self._merge_filter_across_ranks(self._fs_start)
        b = Batch(self.N, self.obs, self.act, self.prob, self.rew, self.flags, self.ep_t, T=self.T, E=self.E)
        b.n_global = self.N_global
        b.rows_owner, b.rows_gen = self, self.rows_gen
        if not self.layered and self.persistent:
            b.abort, b.abort_msg = self.status, self.ABORT_MSG
        return b

    # ------------------------------------------------------------ filter state
    def _merge_filter_across_ranks(self, fs_start):
        s0 = fs_start.double().cpu().numpy()
        s1 = self.filter_state[:self.FS].double().cpu().numpy()
        out = merge_filter_deltas(s0, s1, self.comm)
        self.filter_state[:self.FS].copy_(torch.as_tensor(out))

    def filter_stats(self):
        """(n, mean[obs], var[obs]), (n_rew, mean_rew, var_rew) of the running stats."""
        s = self.filter_state[:self.FS].cpu().numpy()
        D = (self.FS - 2) // 2
        n, nr = s[0], s[1]
        M, S = s[2:2 + D], s[2 + D:2 + 2 * D]
        var_o = S[:D - 1] / (n - 1) if n > 1 else M[:D - 1] ** 2
        var_r = S[D - 1] / (nr - 1) if nr > 1 else M[D - 1] ** 2
        return (n, M[:D - 1].copy(), var_o), (nr, M[D - 1], var_r)

    # ------------------------------------------------------------ episode stats
    def episode_stats(self, batch):
        """add_episode_stats scalars (core.py:31-44), reduced on device and over ranks."""
        return self.episode_stats_finish(self.episode_stats_launch(batch))

    def episode_stats_launch(self, batch):
        """The device half: per-episode sums / maxima reduced on device and over ranks,
        returned as a device tensor (no host sync; the pipelined loop reads it later)."""
        call("mrl_episode_stats", ptr(batch.rew), ptr(batch.flags), batch.T, batch.E, ptr(self._ep_out),
             ptr(self._ep_ws), stream())
        # [6]: the rollout's abort status rides along (summed over ranks: any rank's abort)
        v = torch.cat([self._ep_out[:6], self.status.double()])
        if self.comm.enabled:
            mx = v[[3, 5]].clone()
            self.comm.allreduce_(v)
            torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX, group=self.comm.group)
            v[3], v[5] = mx[0], mx[1]
        return v

    @classmethod
    def episode_stats_finish(cls, v):
        cnt, sr, sr2, mr, sl, ml, abort = (float(x) for x in v.cpu().numpy())
        if abort != 0:
            raise _lib.MrlError(cls.ABORT_MSG)
        mean = sr / cnt
        return dict(NumEpBatch=int(cnt), EpRewMean=mean,
                    EpRewSEM=float(np.sqrt(max(sr2 / cnt - mean * mean, 0.0)) / np.sqrt(cnt)),
                    EpRewMax=mr, EpLenMean=sl / cnt, EpLenMax=ml, RewPerStep=sr / sl)
