"""Agent zoo (`agentzoo.py` of the reference) -- the plug-in layer selected by
``--agent modular_rl_amd.agentzoo.TrpoAgent``.

``TrpoAgent(ob_space, ac_space, usercfg)`` keeps the reference constructor and
``options`` (MLP + PG + TRPO + FILTER), exposes ``act / obfilt / rewfilt /
get_flat / set_from_flat / baseline / updater`` and adds ``make_collector`` for
the lock-step device collector.  Nets are device ``MlpNet`` s (flat fp32 theta)
instead of Keras models; the ZFilter state lives on the device inside the
collector.
"""
import numpy as np

from . import _lib
from .collector import Collector
from .core import PG_OPTIONS, Categorical, DiagGauss, StochPolicyMLP, horizon_of
from .dist import Comm
from .envs import Box, Discrete
from .filters import DeviceZFilter
from .misc_utils import IDENTITY, comma_sep_ints, update_default_config
from .nets import check_hid_sizes, glorot_init, make_net
from .ppo import PpoLbfgsUpdater, PpoSgdUpdater
from .trpo import TrpoUpdater
from .vf import NnVf

MLP_OPTIONS = [
    ("hid_sizes", comma_sep_ints, [64, 64], "Sizes of hidden layers of MLP"),
    ("activation", str, "tanh", "nonlinearity"),
    ("mlp_impl", str, "auto", "HIP MLP path: auto (fused 64-wide kernels when the shape allows), fused, layered"),
    ("mlp_dtype", str, "fp32", "MFMA operand precision of every MLP pass: fp32 (exact, the parity dtype) or "
                               "bf16 (bf16 operands, f32 accumulation: throughput mode)"),
]

FILTER_OPTIONS = [
    ("filter", int, 1, "Whether to do a running average filter of the incoming observations and rewards"),
]


def make_mlps(ob_space, ac_space, cfg, comm=None, seed=0):
    """Policy + value nets (`agentzoo.py:25-60`): tanh MLP, softmax / DiagGauss head,
    last policy kernel x0.1; the VF takes obs + the t/timestep_limit feature."""
    assert isinstance(ob_space, Box)
    if cfg["activation"] != "tanh":
        raise _lib.MrlError("only activation=tanh is implemented on the HIP path")
    hid = check_hid_sizes(cfg["hid_sizes"])
    impl = cfg.get("mlp_impl", "auto")
    dtype = cfg.get("mlp_dtype", "fp32")
    rng = np.random.default_rng(seed)
    if isinstance(ac_space, Box):
        outdim, head, probtype = ac_space.shape[0], _lib.HEAD_GAUSS, DiagGauss(ac_space.shape[0])
    else:
        outdim, head, probtype = ac_space.n, _lib.HEAD_SOFTMAX, Categorical(ac_space.n)
    nin = ob_space.shape[0]
    net = make_net(nin, outdim, head, hid, impl=impl, dtype=dtype)
    net.set_flat(glorot_init(rng, nin, outdim, head, hid))
    policy = StochPolicyMLP(net, probtype)
    vfnet = make_net(nin + 1, 1, _lib.HEAD_LINEAR, hid, impl=impl, dtype=dtype)
    vfnet.set_flat(glorot_init(rng, nin + 1, 1, _lib.HEAD_LINEAR, hid))
    baseline = NnVf(vfnet, cfg["timestep_limit"], dict(mixfrac=0.1), comm=comm)
    return policy, baseline


class AgentWithPolicy:
    """`agentzoo.py:97-114`."""

    def __init__(self, policy, obfilter, rewfilter):
        self.policy = policy
        self.obfilter = obfilter
        self.rewfilter = rewfilter
        self.stochastic = True

    def set_stochastic(self, stochastic):
        self.stochastic = stochastic

    def act(self, ob_no):
        return self.policy.act(ob_no, stochastic=self.stochastic)

    def get_flat(self):
        return self.policy.get_flat()

    def set_from_flat(self, th):
        return self.policy.set_from_flat(th)

    def obfilt(self, ob):
        return self.obfilter(ob)

    def rewfilt(self, rew):
        return self.rewfilter(rew)


class TrpoAgent(AgentWithPolicy):
    options = MLP_OPTIONS + PG_OPTIONS + TrpoUpdater.options + FILTER_OPTIONS
    updater_cls = TrpoUpdater

    def __init__(self, ob_space, ac_space, usercfg, comm=None):
        cfg = update_default_config(self.options, usercfg)
        if not cfg["timestep_limit"]:
            cfg["timestep_limit"] = (usercfg or {}).get("timestep_limit") or 1000
        self.cfg = cfg
        self.comm = comm if comm is not None else Comm()
        seed = int((usercfg or {}).get("seed", 0))
        self.seed = seed
        policy, self.baseline = make_mlps(ob_space, ac_space, cfg, comm=self.comm, seed=seed)
        self.updater = self.updater_cls(policy, cfg, comm=self.comm)
        self._collectors = {}
        self._pending_state = None  # filter / RNG state from load_snapshot, applied to the first collector
        if cfg["filter"]:
            obfilter = DeviceZFilter(self, "obs", clip=5)
            rewfilter = DeviceZFilter(self, "rew", demean=False, clip=10)
        else:
            obfilter = rewfilter = IDENTITY
        AgentWithPolicy.__init__(self, policy, obfilter, rewfilter)

    # ---- device collection
    def make_collector(self, env, cfg=None, n_envs=None, horizon=None, timestep_limit=None):
        cfg = self.cfg if cfg is None else cfg
        E = int(n_envs or cfg.get("n_envs", 1) or 1)
        T = int(horizon or horizon_of(cfg))
        limit = int(timestep_limit or cfg["timestep_limit"] or env.spec.max_episode_steps)
        key = (env.spec.id, E, T, limit)
        if key not in self._collectors:
            col = Collector(env, self.policy, E, T, limit, filter=self.cfg["filter"], seed=self.seed, comm=self.comm,
                            use_graph=bool(cfg.get("use_graph", self.cfg.get("use_graph", 1))))
            shared = self._filter_owner()
            if shared is not None:  # one running stat per agent
                col.filter_state = shared.filter_state
            elif self._pending_state:
                from .checkpoint import apply_collector_state
                apply_collector_state(col, self._pending_state)
                self._pending_state = None
            self._collectors[key] = col
        return self._collectors[key]

    def path_collector(self, env, timestep_limit):
        return self.make_collector(env, n_envs=1, horizon=int(timestep_limit), timestep_limit=timestep_limit)

    def _filter_owner(self):
        for c in self._collectors.values():
            return c
        return None


class PpoLbfgsAgent(TrpoAgent):
    """`agentzoo.py:134-141`: PPO with the L-BFGS penalty updater."""
    options = MLP_OPTIONS + PG_OPTIONS + PpoLbfgsUpdater.options + FILTER_OPTIONS
    updater_cls = PpoLbfgsUpdater


class PpoSgdAgent(TrpoAgent):
    """`agentzoo.py:143-150`: PPO with minibatch Adam."""
    options = MLP_OPTIONS + PG_OPTIONS + PpoSgdUpdater.options + FILTER_OPTIONS
    updater_cls = PpoSgdUpdater
