"""Training-loop layer with the reference's names (`core.py` of ddlau/modular_rl).

The loop ``run_policy_gradient_algorithm`` (`core.py:118-171`) keeps its contract
(``callback(stats)`` once per iteration with EpRewMean / vf_* / pol_* /
TimeElapsed keys) but each stage is device-resident:

  rollouts            Collector.collect()          fused lock-step HIP rollout
  compute_advantage   NnVf forward + mrl_gae + global standardisation
  VF update           NnVf.fit_batch               L-BFGS with device loss/grad
  policy update       TrpoUpdater.update           device CG / line search

The per-path API (``rollout``, ``do_rollouts_serial``, ``compute_advantage(vf,
paths, ...)``, ``agent.updater(paths)``) is kept for compatibility and runs the
same kernels on E = 1.
"""
import contextlib
import os
import time
from collections import OrderedDict
from importlib import import_module

import numpy as np
import torch

from . import _lib, timing
from ._lib import call, ptr, stream
from .collector import Batch, Collector
from .dist import Comm
from .checkpoint import capture_host_state, capture_state
from .misc_utils import update_default_config
from .vf import LbfgsOptimizer, NnRegression, NnVf  # noqa: F401  (reference names live in core)

concat = np.concatenate


def get_agent_cls(name):
    """`core.py:20-24`."""
    p, m = name.rsplit(".", 1)
    mod = import_module(p)
    return getattr(mod, m)


def add_episode_stats(stats, paths):
    """`core.py:31-44` (per-path form)."""
    reward_key = "reward_raw" if "reward_raw" in paths[0] else "reward"
    episoderewards = np.array([path[reward_key].sum() for path in paths])
    pathlengths = np.array([pathlength(path) for path in paths])
    stats["EpisodeRewards"] = episoderewards
    stats["EpisodeLengths"] = pathlengths
    stats["NumEpBatch"] = len(episoderewards)
    stats["EpRewMean"] = episoderewards.mean()
    stats["EpRewSEM"] = episoderewards.std() / np.sqrt(len(paths))
    stats["EpRewMax"] = episoderewards.max()
    stats["EpLenMean"] = pathlengths.mean()
    stats["EpLenMax"] = pathlengths.max()
    stats["RewPerStep"] = episoderewards.sum() / pathlengths.sum()


def add_prefixed_stats(stats, prefix, d):
    for k, v in d.items():
        stats[prefix + "_" + k] = v


# ================================================================ advantage
class _GaeWorkspace:
    """mrl_gae's own workspace (zeroed once: it carries a completion counter between calls)
    and the moments passes' scratch, kept apart."""

    def __init__(self):
        self.ws = self.ws_gae = None
        self.moments = None

    def get(self, T, E, device):
        lib = _lib.load()
        nbytes = int(lib.mrl_moments_workspace_bytes(int(T * E)))
        gbytes = int(lib.mrl_gae_workspace_bytes(int(T), int(E)))
        if (self.ws is None or self.ws.numel() < nbytes or self.ws_gae.numel() < gbytes
                or self.ws.device != device):
            self.ws = torch.zeros(nbytes, dtype=torch.uint8, device=device)
            self.ws_gae = torch.zeros(gbytes, dtype=torch.uint8, device=device)
            self.moments = torch.zeros(2, 3, dtype=torch.float64, device=device)  # first pass, centred pass
        return self.ws_gae, self.ws, self.moments


_GAE = _GaeWorkspace()


def gae_scan(batch, gamma, lam):
    """The GAE + discounted-return scan of a time-major batch (mrl_gae: adv / ret rows and
    the first-pass moments into the module workspace) -- compute_advantage_batch's scan,
    also timed on its own by bench.py."""
    ws_gae, _, moments = _GAE.get(batch.T, batch.E, batch.rew.device)
    call("mrl_gae", ptr(batch.rew), ptr(batch.vpred), ptr(batch.flags), int(batch.T), int(batch.E), float(gamma),
         float(lam), ptr(batch.adv), ptr(batch.ret), ptr(moments), ptr(ws_gae), stream())
    return moments


def compute_advantage_batch(vf, batch, gamma, lam, comm=None):
    """Device form of `core.py:63-105` on a time-major batch: baseline forward,
    GAE + discounted return scan (mrl_gae), then standardisation with the global
    (all-rank) mean / std (numpy std, ddof=0, no epsilon)."""
    comm = comm if comm is not None else Comm()
    dev = batch.obs.device
    n = batch.n
    batch.vpred = vf.predict_batch(batch, out=batch.vpred if batch.vpred is not None and batch.vpred.numel() == n
                                   else torch.empty(n, dtype=torch.float32, device=dev))
    if batch.adv is None or batch.adv.numel() != n:
        batch.adv = torch.empty(n, dtype=torch.float32, device=dev)
        batch.ret = torch.empty(n, dtype=torch.float32, device=dev)
    ws, moments = _GAE.get(batch.T, batch.E, dev)[1:]
    timing.start("gae_scan", detail=True)
    gae_scan(batch, gamma, lam)
    timing.stop("gae_scan")
    # numpy's two-pass std (core.py:100-105): global mean first, then the centred sums
    comm.allreduce_(moments[0])
    call("mrl_moments_centered", ptr(batch.adv), None, int(n), ptr(moments[0]), ptr(moments[1]), ptr(ws), stream())
    comm.allreduce_(moments[1])
    call("mrl_standardize", ptr(batch.adv), int(n), ptr(moments[0]), ptr(moments[1]), stream())
    return batch


def compute_advantage(vf, paths, gamma, lam):
    """Per-path API of `core.py:63-105`: fills path["return"], ["baseline"],
    ["advantage"] (standardised over all paths)."""
    dev = vf.net.device
    batch = Batch.from_paths(paths, None, device=dev, need_policy=False)
    compute_advantage_batch(vf, batch, gamma, lam)
    adv = batch.adv.cpu().numpy().astype(np.float64)
    ret = batch.ret.cpu().numpy().astype(np.float64)
    base = batch.vpred.cpu().numpy().astype(np.float64)
    i = 0
    for path in paths:
        L = len(path["reward"])
        path["return"], path["baseline"], path["advantage"] = ret[i:i + L], base[i:i + L], adv[i:i + L]
        i += L


PG_OPTIONS = [
    ("timestep_limit", int, 0, "maximum length of trajectories"),
    ("n_iter", int, 200, "number of batch"),
    ("parallel", int, 0, "collect trajectories in parallel"),
    ("timesteps_per_batch", int, 100, ""),
    ("gamma", float, 0.99, "discount"),
    ("lam", float, 1.0, "lambda parameter from generalized advantage estimation"),
    # MI355X build: lock-step batched collection
    ("n_envs", int, 1, "envs stepped in lock-step per GPU"),
    ("horizon", int, 0, "steps per env per iteration (0: ceil(timesteps_per_batch / n_envs))"),
    ("use_graph", int, 1, "replay the rollout's per-step launches from one captured hipGraph"),
    ("pipeline", int, 1, "run the VF fit of iteration k beside the rollout of iteration k+1 on disjoint CUs"),
]


def horizon_of(cfg):
    h = int(cfg.get("horizon", 0) or 0)
    if h <= 0:
        h = -(-int(cfg["timesteps_per_batch"]) // int(cfg.get("n_envs", 1) or 1))
    return max(h, 1)


def run_policy_gradient_algorithm(env, agent, usercfg=None, callback=None):
    """`core.py:118-171`: rollouts -> advantage -> VF fit -> TRPO update -> callback(stats)."""
    cfg = update_default_config(PG_OPTIONS, usercfg)
    cfg.update(usercfg or {})
    if cfg["parallel"]:
        raise NotImplementedError("parallel rollouts: launch one process per GPU with torchrun instead")
    comm = agent.comm
    collector = agent.make_collector(env, cfg)
    runner = IterationRunner(agent, collector, cfg, comm, pipeline=bool(cfg["pipeline"]))
    tstart = time.time()

    def emit(stats):
        stats["TimeElapsed"] = time.time() - tstart
        if callback:
            callback(stats)
        # the runner's capture describes the iteration just reported; a snapshot taken
        # after this callback must read the live state
        agent._snapshot_capture = None

    with runner.loop_stream():
        for i in range(cfg["n_iter"]):
            done = runner.step(prelaunch_next=i + 1 < cfg["n_iter"])
            if done is not None:
                emit(done)
        done = runner.drain()
    if done is not None:
        emit(done)


LAYERED_ROLLOUT_CUS = int(os.environ.get("MRL_LAYERED_ROLLOUT_CUS", "64"))


def rollout_cus_needed(collector):
    """CUs the rollout's step chain wants to itself: the fused step kernel one block per
    CU (NB); Humanoid's wave-per-env step one wave per SIMD (E / 4 CUs); other layered
    rollouts LAYERED_ROLLOUT_CUS for their GEMM tiles."""
    if getattr(collector, "wave_per_env", False):
        return -(-collector.E // 4)
    return LAYERED_ROLLOUT_CUS if collector.layered else collector.NB


def rollout_cu_split(n_rollout, n_cus):
    """(rollout CUs, fit CUs) for the pipelined loop, or None when the rollout needs
    too many CUs for a split to pay.  The fused rollout step kernel runs one block per
    CU (one wave per SIMD: its latency chain wants no co-resident waves), so it gets
    as many CUs as it has blocks; the layered rollout's per-step GEMMs over E rows use
    a few dozen tiles and get LAYERED_ROLLOUT_CUS.  The VF fit gets every other CU."""
    if n_rollout <= 0 or 2 * n_rollout > n_cus:
        return None
    r = list(range(n_rollout))
    # MRL_FIT_CUS caps the fit's share (diagnostic A/B: the fit beside the rollout slows
    # the rollout's latency chain through shared clock / memory)
    cap = int(os.environ.get("MRL_FIT_CUS", "0"))
    hi = n_cus if cap <= 0 else min(n_cus, n_rollout + cap)
    return r, list(range(n_rollout, hi))


def fit_comm_for(comm, beside_rollout):
    """The Comm the VF fit reduces over: a host (gloo) group when the fit runs beside the
    rollout on more than one rank, else the iteration's own (RCCL) Comm."""
    return comm.host() if beside_rollout and comm.enabled and comm.world > 1 else comm


class IterationRunner:
    """One iteration of `core.py:146-157` per ``step()``: rollout -> compute_advantage
    -> VF fit -> policy update -> stats.

    ``pipeline``: the VF fit of iteration k is deferred and run on a CU-masked stream
    while iteration k+1's rollout runs on the disjoint CU set (streams.masked_stream).
    The dependencies are exactly the sequential ones -- the rollout of k+1 needs the
    policy after update k (not the VF); compute_advantage of k+1 needs the VF after
    fit k (so it waits for the fit); fit k reads only iteration k's features, target,
    returns and V_old, which nothing of iteration k+1 overwrites before it -- so every
    kernel sees the same inputs as in the reference order and the results are
    bit-identical to ``pipeline=False``.  ``step()`` returns the stats of the iteration
    whose VF fit finished during it (pipelined: the previous one) and ``drain()`` the
    last one."""

    def __init__(self, agent, collector, cfg, comm=None, pipeline=True):
        self.agent, self.col, self.cfg = agent, collector, cfg
        self.comm = comm if comm is not None else Comm()
        self.pending = None
        self._prelaunched = None  # events of a rollout issued by the previous step
        self.pipeline = False
        self.last_phase_events = None
        self.record_phases = False
        self.last_drain_events = {}
        self._vorder = None  # streams.ValueOrder of the pipelined loop (set below)
        if torch.cuda.is_available():
            from . import streams
            need = rollout_cus_needed(collector)
            split = rollout_cu_split(need, streams.cu_count())
            # the VF passes are sized for the fit's CU set in BOTH orders: their partial
            # sums follow the grid, and the two orders stay bit-identical
            vf_net = getattr(getattr(agent, "baseline", None), "net", None)
            if split is not None and hasattr(vf_net, "size_for_cus"):
                vf_net.size_for_cus(len(split[1]))
            # C5 (r04x, Humanoid bf16, 1024 envs): 487 -> 450 ms per iteration at 3 steps
            # (the rollout 235 -> 289 ms beside the fit, the 124 ms fit hidden); MRL_COSCHED_FIT=0
            # keeps the fit after the rollout
            cosched_ok = (split is None and getattr(collector, "wave_per_env", False)
                          and os.environ.get("MRL_COSCHED_FIT", "1") == "1")
            cosched = pipeline and cosched_ok
            if cosched_ok and hasattr(vf_net, "lds_limit"):
                # in BOTH orders (its kernels' choice must not depend on the order):
                # MRL_COSCHED_LDS bytes of LDS per GEMM block, 0 = no limit (r04i: a 64 KB
                # cap slowed the fit 15 ms and not the rollout's slowdown; off)
                vf_net.lds_limit = int(os.environ.get("MRL_COSCHED_LDS", "0"))
            if cosched:
                # Humanoid's wave-per-env step wants every CU (E / 4), so no disjoint split:
                # the fit of iteration k shares the CUs with the rollout of k+1 (two plain
                # streams; one wave per SIMD in the step kernel leaves issue slots free)
                # MRL_COSCHED_PRIO (default 1; r04j: +1 %, within box noise): the rollout
                # stream at high priority, its per-step blocks dispatched ahead of the fit's
                prio = -1 if os.environ.get("MRL_COSCHED_PRIO", "1") == "1" else 0
                self.rollout_stream = torch.cuda.Stream(priority=prio)
                self.fit_stream = torch.cuda.Stream()
            if pipeline and (split is not None or cosched):
                if not cosched:
                    self.rollout_stream = streams.masked_stream(split[0])
                    self.fit_stream = streams.masked_stream(split[1])
                # the iteration's own work runs on a non-blocking stream: an event recorded
                # on the legacy NULL stream would wait for the rollout stream's work and
                # serialise the fit behind it
                self.main_stream = torch.cuda.Stream()
                self.pipeline = True
                if os.environ.get("MRL_XSTREAM_EVENT", "0") != "1":
                    self._vorder = streams.ValueOrder()
                # data-parallel: the fit's per-evaluation reductions go over a host group
                # while it overlaps the persistent rollout (RCCL's kernels would land on
                # the rollout's CUs and delay its hand-off polls).  The
                # co-scheduled Humanoid rollout is step launches with no cross-block
                # polling, so its fit keeps RCCL (2.9 MB gradients per evaluation)
                reg = getattr(getattr(agent, "baseline", None), "reg", None)
                if reg is not None and hasattr(reg, "set_comm"):
                    reg.set_comm(fit_comm_for(getattr(reg, "comm", self.comm), not cosched))

    @staticmethod
    def _stats(ep, vf_stats, pol_stats):
        stats = OrderedDict()
        stats.update(ep)
        add_prefixed_stats(stats, "vf", vf_stats)
        add_prefixed_stats(stats, "pol", pol_stats)
        return stats

    def _order(self, producer, consumer):
        """consumer's later work after producer's prior work: on a memory value (the
        rollout <-> iteration streams; streams.ValueOrder, ~10 us less per crossing than
        an event) unless MRL_XSTREAM_EVENT=1."""
        if self._vorder is None:
            return consumer.wait_stream(producer)
        self._vorder.order(producer, consumer)

    def _event(self):
        """A phase boundary's timing event -- only on the iterations timing samples (bench.py's
        timed region) or when record_phases is set: each one is a queue marker that delays
        the next kernel by ≈6 µs (modular_rl_amd/timing.py)."""
        if not (self.record_phases or timing.detail_now()):
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _on_main(self, fn):
        if not self.pipeline:
            return fn()
        caller = torch.cuda.current_stream()
        self.main_stream.wait_stream(caller)
        with torch.cuda.stream(self.main_stream):
            out = fn()
        caller.wait_stream(self.main_stream)
        return out

    def loop_stream(self):
        """Context for a loop of step() calls: the iteration's own stream (pipelined).
        Called from the legacy default stream, step() orders itself after it by an event
        on that stream -- and an operation on the legacy stream also waits for all work of
        the blocking streams, among them the CU-masked rollout stream (hipExtStream-
        CreateWithCUMask takes no flags): a rollout prelaunched by the previous step would
        then hold back this step's VF fit until it finished (measured: the fit serialised
        behind the rollout, 41.2 instead of 33 ms per Hopper iteration).  Inside this
        context the caller IS the iteration's stream and no legacy-stream operation is
        issued."""
        if not self.pipeline:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.main_stream)

    def step(self, prelaunch_next=False):
        """One iteration.  ``prelaunch_next``: another step follows, so the next
        iteration's rollout is issued as soon as the policy update has set the new theta
        (TrpoUpdater.after_theta) -- the stats, the snapshot capture and the loop's host
        Python then run under that rollout instead of in front of it."""
        return self._on_main(lambda: self._step(prelaunch_next))

    def _launch_rollout(self, noise_ready=False):
        """Issue one iteration's rollout (the noise fill and the step chain); its events.
        ``noise_ready``: the noise fill was issued already (under the update's readback)."""
        col, ev = self.col, {}
        ev["rollout0"] = self._event()
        if self.pipeline:
            main = torch.cuda.current_stream()
            if not noise_ready:
                col.fill_noise()  # one wide kernel: on every CU, ahead of the step chain
            self._order(main, self.rollout_stream)
            with torch.cuda.stream(self.rollout_stream):
                col.launch(fill_noise=False)
                ev["rollout1"] = self._event()
        else:
            col.launch()
            ev["rollout1"] = self._event()
        return ev

    def _step(self, prelaunch_next=False):
        cfg, agent, col = self.cfg, self.agent, self.col
        main = torch.cuda.current_stream()
        ev = self._prelaunched if getattr(self, "_prelaunched", None) is not None else self._launch_rollout()
        self._prelaunched = None
        done = None
        if self.pipeline:
            if self.pending is not None:
                done = self._fit_pending(self.fit_stream, ev)
            self._order(self.rollout_stream, main)
        batch = col.finish()
        self.last_batch = batch
        ev["adv0"] = self._event()
        compute_advantage_batch(agent.baseline, batch, cfg["gamma"], cfg["lam"], self.comm)
        ev["adv1"] = self._event()
        # the episode statistics read this batch's rewards / flags: issued before the next
        # rollout (launched from the update below) can overwrite them
        ep_dev = col.episode_stats_launch(batch)
        vf_stats = None
        if not self.pipeline:
            ev["vf0"] = self._event()
            vf_stats = agent.baseline.fit_batch(batch)
            ev["vf1"] = self._event()
        ev["upd0"] = self._event()
        post = {}

        def after_theta():
            """The next iteration's theta is final: snapshot capture (the filter state and
            RNG counters the next rollout advances), then that rollout."""
            if "cap" in post:
                return
            ev["upd1"] = self._event()
            # pipelined: the VF of this iteration is fitted during the next step and added
            # to the capture then; in order it is final already
            # the state the next rollout advances: taken under the readback already when
            # before_readback ran (nothing changes it in between), else here
            early = post.pop("cap_early", None)
            post["cap"] = early if early is not None else capture_state(agent, with_vf=not self.pipeline,
                                                                       host=False, theta=False)
            if prelaunch_next:
                self._prelaunched = self._launch_rollout(noise_ready=post.pop("noise", False))
            # theta (the rollout only reads it), numpy's RNG and the updater's arrays:
            # nothing the rollout writes, so taken under it (off the update-to-rollout seam)
            post["cap"]["policy/theta"] = agent.policy.net.theta.detach().clone()
            post["cap"].update(capture_host_state(agent))

        def before_readback():
            """The next rollout's noise (a function of the collector's iteration counter,
            which this iteration's rollout has advanced already) and the snapshot copies of
            the state that rollout advances (filter state, RNG counters: final since this
            iteration's rollout): issued behind the update's readback, they run while the
            host decides the line search."""
            if prelaunch_next and self.pipeline and "cap" not in post:
                col.fill_noise()
                post["noise"] = True
                post["cap_early"] = capture_state(agent, with_vf=False, host=False, theta=False)

        upd = agent.updater
        upd.after_theta = after_theta
        upd.before_readback = before_readback
        try:
            pol_stats = upd.update(batch)
        finally:
            upd.after_theta = None
            upd.before_readback = None
        after_theta()  # updaters without the hook
        if self.pipeline:
            # read back with the deferred VF fit's stats (no host sync here); the state at
            # the end of this iteration (the VF after its fit is added then) is captured
            # for snapshots taken in the callback that reports it
            self.pending = (batch, ep_dev, pol_stats, post["cap"])
        else:
            # a snapshot taken in this iteration's callback reads the state at its end, not
            # the live one (the next rollout may already be running)
            agent._snapshot_capture = post["cap"]
            done = self._stats(col.episode_stats_finish(ep_dev), vf_stats, pol_stats)
        self.last_phase_events = ev
        return done

    def _fit_pending(self, fit_stream, ev):
        batch, ep_dev, pol_stats, cap = self.pending
        self.pending = None
        main = torch.cuda.current_stream()
        vf_net = self.agent.baseline.net
        if fit_stream is None:
            ev["vf0"] = self._event()
            vf_stats = self.agent.baseline.fit_batch(batch)
            ev["vf1"] = self._event()
            cap["vf/theta"] = vf_net.theta.detach().clone()
        else:
            fit_stream.wait_stream(main)
            with torch.cuda.stream(fit_stream):
                ev["vf0"] = self._event()
                vf_stats = self.agent.baseline.fit_batch(batch)
                ev["vf1"] = self._event()
                cap["vf/theta"] = vf_net.theta.detach().clone()
            main.wait_stream(fit_stream)
        self.agent._snapshot_capture = cap
        return self._stats(self.col.episode_stats_finish(ep_dev), vf_stats, pol_stats)

    def drain(self):
        """Fit the deferred VF of the last iteration (on all CUs) and return its stats."""
        if self.pending is None:
            return None
        ev = {}
        done = self._on_main(lambda: self._fit_pending(None, ev))
        self.last_drain_events = ev
        return done


# ================================================================ per-path API
def get_paths(env, agent, cfg, seed_iter):
    if cfg["parallel"]:
        raise NotImplementedError
    return do_rollouts_serial(env, agent, cfg["timestep_limit"], cfg["timesteps_per_batch"], seed_iter)


def rollout(env, agent, timestep_limit):
    """One episode (`core.py:182-207`) through the device collector with E = 1."""
    col = agent.path_collector(env, timestep_limit)
    while True:
        paths = col.collect().to_paths()
        if paths:
            return paths[0]


def do_rollouts_serial(env, agent, timestep_limit, n_timesteps, seed_iter):
    """Whole episodes until more than n_timesteps steps (`core.py:210-221`)."""
    paths = []
    timesteps_sofar = 0
    while True:
        next(seed_iter)
        path = rollout(env, agent, timestep_limit)
        paths.append(path)
        timesteps_sofar += pathlength(path)
        if timesteps_sofar > n_timesteps:
            break
    return paths


def pathlength(path):
    return len(path["action"])


# ================================================================ policies / probtypes
class ProbType:
    pass


class Categorical(ProbType):
    """`core.py:339-365` (device math lives in mrl_mlp_rows; this is the host API)."""

    def __init__(self, n):
        self.n = n

    def sample(self, prob):
        cs = np.cumsum(prob, axis=1)
        return np.argmax(cs > np.random.rand(prob.shape[0], 1), axis=1)

    def maxprob(self, prob):
        return prob.argmax(axis=1)


class DiagGauss(ProbType):
    """`core.py:402-438`."""

    def __init__(self, d):
        self.d = d

    def sample(self, prob):
        mean_nd, std_nd = prob[:, :self.d], prob[:, self.d:]
        return np.random.randn(prob.shape[0], self.d).astype(np.float32) * std_nd + mean_nd

    def maxprob(self, prob):
        return prob[:, :self.d]


class StochPolicyMLP:
    """Device replacement of StochPolicyKeras (`core.py:296-336`)."""

    def __init__(self, net, probtype):
        self.net = net
        self._probtype = probtype
        self.discrete = isinstance(probtype, Categorical)

    @property
    def probtype(self):
        return self._probtype

    def act(self, ob, stochastic=True):
        """`core.py:261-267`: single-row forward on device."""
        x = torch.as_tensor(np.asarray(ob, dtype=np.float32)[None]).to(self.net.device)
        prob = self.net.forward(x, 1).cpu().numpy().reshape(1, -1)
        a = self.probtype.sample(prob) if stochastic else self.probtype.maxprob(prob)
        return a[0], {"prob": prob[0]}

    def get_flat(self):
        return self.net.get_flat()

    def set_from_flat(self, th):
        self.net.set_flat(th)
