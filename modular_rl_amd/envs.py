"""Env registry for the device env steppers (replaces ``gym.envs.make``, run_pg.py:85).

The dynamics live in ``csrc/envs.h`` and run inside the fused rollout kernel; this
module only describes them with gym-compatible spaces / spec so that
``TrpoAgent(env.observation_space, env.action_space, cfg)`` and
``env.spec.max_episode_steps`` (run_pg.py:103-108) work unchanged.

* ``CartPole-v0`` -- gym's classic-control CartPole equations, TimeLimit 200.
* ``Hopper-v2``   -- gym's hopper.xml as articulated rigid-body dynamics (obs 11, act 3, TimeLimit 1000);
  MuJoCo is not available, so its dynamics are a stand-in.
* ``Humanoid-v2`` -- Humanoid-v2-SHAPED surrogate (obs 376, act 17 in [-0.4, 0.4],
  TimeLimit 1000); its 376-d obs needs the layered rollout (collector.py).
"""
import numpy as np

from . import _lib


class Box:
    def __init__(self, low, high, shape):
        self.shape = tuple(shape)
        self.low = np.full(self.shape, low, dtype=np.float32)
        self.high = np.full(self.shape, high, dtype=np.float32)

    def __repr__(self):
        return f"Box{self.shape}"


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()

    def __repr__(self):
        return f"Discrete({self.n})"


class EnvSpec:
    def __init__(self, env_id, max_episode_steps):
        self.id = env_id
        self.max_episode_steps = max_episode_steps


REGISTRY = {
    "CartPole-v0": dict(kind=_lib.ENV_CARTPOLE, obs=4, act=2, discrete=True, max_steps=200, obs_high=np.inf),
    "Hopper-v2": dict(kind=_lib.ENV_HOPPER, obs=11, act=3, discrete=False, max_steps=1000, obs_high=np.inf),
    "Humanoid-v2": dict(kind=_lib.ENV_HUMANOID, obs=376, act=17, discrete=False, max_steps=1000, obs_high=np.inf,
                        act_high=0.4),
}


class DeviceEnv:
    """Description of a batched device env (the state itself lives in a Collector)."""

    def __init__(self, env_id):
        if env_id not in REGISTRY:
            raise ValueError(f"unknown env {env_id!r}; available: {sorted(REGISTRY)}")
        r = REGISTRY[env_id]
        self.kind = r["kind"]
        self.obs_dim = r["obs"]
        self.observation_space = Box(-r["obs_high"], r["obs_high"], (r["obs"],))
        ah = r.get("act_high", 1.0)
        self.action_space = Discrete(r["act"]) if r["discrete"] else Box(-ah, ah, (r["act"],))
        self.discrete = r["discrete"]
        self.act_dim = r["act"]
        self.spec = EnvSpec(env_id, r["max_steps"])

    def close(self):
        pass


def make(env_id):
    return DeviceEnv(env_id)
