"""Env dynamics restated in numpy float64 -- TEST INFRASTRUCTURE (oracle).

The reference builds its envs with ``gym.envs.make(args.env)`` (`run_pg.py:85`)
and steps them through the 4-tuple API (`core.py:186,197`); gym and MuJoCo are
not vendored and are absent here, so env dynamics are **parity unpinned**:

* ``cartpole_*`` restates gym's CartPole-v0 equations (Euler, tau=0.02,
  force 10, 12-degree / 2.4 thresholds, reward 1 per step, TimeLimit 200).
* ``hopper_*`` is a *surrogate* with Hopper-v2's interface (11-d obs =
  qpos[1:] ++ clip(qvel, -10, 10), 3-d action in [-1, 1] with gear 200,
  frame_skip 4 x dt 0.002, reward = forward velocity + 1 - 1e-3 |a|^2, the
  Hopper-v2 health test, TimeLimit 1000).  Its planar leg dynamics are a
  cost-representative stand-in for MuJoCo, not MuJoCo.

Every function here is mirrored operation-for-operation by the HIP env kernels
in ``modular_rl_amd/csrc/envs.h`` (compiled with fp-contract off) so the GPU
collector can be checked against it in float64.
"""
import numpy as np

# ---------------------------------------------------------------- CartPole-v0
CP_GRAVITY = 9.8
CP_MASSCART = 1.0
CP_MASSPOLE = 0.1
CP_TOTAL_MASS = CP_MASSPOLE + CP_MASSCART
CP_LENGTH = 0.5
CP_POLEMASS_LENGTH = CP_MASSPOLE * CP_LENGTH
CP_FORCE_MAG = 10.0
CP_TAU = 0.02
CP_THETA_THRESHOLD = 12 * 2 * np.pi / 360
CP_X_THRESHOLD = 2.4


def cartpole_reset(u):
    """u: [..., 4] uniforms in [0,1) -> state U(-0.05, 0.05)^4."""
    return u * 0.1 - 0.05


def cartpole_obs(s):
    return s.copy()


def cartpole_step(s, a):
    """s: [E,4] float64, a: [E] int -> (s', reward, done)."""
    x, x_dot, theta, theta_dot = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    force = np.where(a == 1, CP_FORCE_MAG, -CP_FORCE_MAG)
    costheta = np.cos(theta)
    sintheta = np.sin(theta)
    temp = (force + CP_POLEMASS_LENGTH * theta_dot * theta_dot * sintheta) / CP_TOTAL_MASS
    thetaacc = (CP_GRAVITY * sintheta - costheta * temp) / (
        CP_LENGTH * (4.0 / 3.0 - CP_MASSPOLE * costheta * costheta / CP_TOTAL_MASS))
    xacc = temp - CP_POLEMASS_LENGTH * thetaacc * costheta / CP_TOTAL_MASS
    x = x + CP_TAU * x_dot
    x_dot = x_dot + CP_TAU * xacc
    theta = theta + CP_TAU * theta_dot
    theta_dot = theta_dot + CP_TAU * thetaacc
    s2 = np.stack([x, x_dot, theta, theta_dot], axis=1)
    done = (x < -CP_X_THRESHOLD) | (x > CP_X_THRESHOLD) | (theta < -CP_THETA_THRESHOLD) | (theta > CP_THETA_THRESHOLD)
    rew = np.ones_like(x)
    return s2, rew, done


# ---------------------------------------------------------------- Hopper surrogate
HP_DT = 0.002
HP_FRAME_SKIP = 4
HP_GEAR = 200.0
HP_GRAV = 9.81
HP_MASS = 3.5
HP_I_ROOT = 2.0
HP_I = (4.0, 3.0, 1.5)
HP_K = (30.0, 30.0, 20.0)
HP_C = (8.0, 6.0, 4.0)
HP_LO = (-2.61799, -2.61799, -0.785398)
HP_HI = (0.0, 0.0, 0.785398)
HP_L_TORSO = 0.2
HP_L_THIGH = 0.45
HP_L_LEG = 0.5
HP_FOOT_R = 0.1
HP_KC = 5000.0
HP_CC = 60.0
HP_MU = 0.9
HP_VMAX = 50.0


def hopper_reset(u):
    """u: [..., 12] uniforms -> (qpos[...,6], qvel[...,6]); init_qpos = (0, 1.25, 0, 0, 0, 0)."""
    qpos = u[..., :6] * 0.01 - 0.005
    qpos[..., 1] = qpos[..., 1] + 1.25
    qvel = u[..., 6:] * 0.01 - 0.005
    return qpos, qvel


def hopper_obs(qpos, qvel):
    return np.concatenate([qpos[:, 1:], np.clip(qvel, -10.0, 10.0)], axis=1)


def _hopper_substep(q, v, tau):
    x, z, ar, a1, a2, a3 = (q[:, i] for i in range(6))
    vx, vz, var_, v1, v2, v3 = (v[:, i] for i in range(6))
    p1 = ar + a1
    p2 = p1 + a2
    w1 = var_ + v1
    w2 = w1 + v2
    s0, c0 = np.sin(ar), np.cos(ar)
    s1, c1 = np.sin(p1), np.cos(p1)
    s2, c2 = np.sin(p2), np.cos(p2)
    # leg tip (contact point) by planar forward kinematics from the root
    fx = x + HP_L_TORSO * s0 + HP_L_THIGH * s1 + HP_L_LEG * s2
    fz = z - HP_L_TORSO * c0 - HP_L_THIGH * c1 - HP_L_LEG * c2
    fvx = vx + HP_L_TORSO * c0 * var_ + HP_L_THIGH * c1 * w1 + HP_L_LEG * c2 * w2
    fvz = vz + HP_L_TORSO * s0 * var_ + HP_L_THIGH * s1 * w1 + HP_L_LEG * s2 * w2
    pen = HP_FOOT_R - fz
    fn = np.where(pen > 0.0, np.maximum(HP_KC * pen - HP_CC * fvz, 0.0), 0.0)
    ft = -HP_MU * fn * np.tanh(fvx / 0.05) * (1.0 - 0.5 * np.abs(np.sin(a3)))
    # accelerations
    ax = ft / HP_MASS
    az = fn / HP_MASS - HP_GRAV
    tq_root = (fx - x) * fn - (fz - z) * ft
    hx = x + HP_L_TORSO * s0
    hz = z - HP_L_TORSO * c0
    kx = hx + HP_L_THIGH * s1
    kz = hz - HP_L_THIGH * c1
    tq1 = (fx - hx) * fn - (fz - hz) * ft
    tq2 = (fx - kx) * fn - (fz - kz) * ft
    aar = (0.05 * tq_root - tau[:, 0] * 0.1 - 1.0 * var_) / HP_I_ROOT
    aa1 = (tau[:, 0] - HP_K[0] * a1 - HP_C[0] * v1 + 0.05 * tq1) / HP_I[0]
    aa2 = (tau[:, 1] - HP_K[1] * a2 - HP_C[1] * v2 + 0.05 * tq2) / HP_I[1]
    aa3 = (tau[:, 2] - HP_K[2] * a3 - HP_C[2] * v3 - 0.02 * ft) / HP_I[2]
    acc = np.stack([ax, az, aar, aa1, aa2, aa3], axis=1)
    v = np.clip(v + HP_DT * acc, -HP_VMAX, HP_VMAX)
    q = q + HP_DT * v
    # joint limits: clamp position, kill the velocity into the limit
    for j, lo, hi in zip((3, 4, 5), HP_LO, HP_HI):
        over = q[:, j] > hi
        under = q[:, j] < lo
        q[:, j] = np.where(over, hi, np.where(under, lo, q[:, j]))
        v[:, j] = np.where(over | under, 0.0, v[:, j])
    return q, v


def hopper_step(qpos, qvel, a):
    """qpos,qvel: [E,6] float64; a: [E,3] -> (qpos', qvel', reward, done)."""
    a = np.asarray(a, dtype=np.float64)
    ac = np.clip(a, -1.0, 1.0)
    tau = HP_GEAR * ac
    x_before = qpos[:, 0].copy()
    q, v = qpos.copy(), qvel.copy()
    for _ in range(HP_FRAME_SKIP):
        q, v = _hopper_substep(q, v, tau)
    x_after = q[:, 0]
    rew = (x_after - x_before) / (HP_DT * HP_FRAME_SKIP) + 1.0 - 1e-3 * (a * a).sum(axis=1)
    s = np.concatenate([q, v], axis=1)
    healthy = np.isfinite(s).all(axis=1) & (np.abs(s[:, 2:]) < 100).all(axis=1) & (q[:, 1] > 0.7) & (np.abs(q[:, 2]) < 0.2)
    return q, v, rew, ~healthy


ENV_SPECS = {
    # id: (obs_dim, act_dim or n, discrete, max_episode_steps)
    "CartPole-v0": (4, 2, True, 200),
    "Hopper-v2": (11, 3, False, 1000),
}
