// Batched env dynamics on device (fp64, struct-of-arrays state), operation-for-
// operation twins of oracle/envs.py.  FMA contraction is disabled so the results
// follow the same rounding sequence as the numpy oracle.
//
//  * CartPole-v0: gym's classic-control equations (Euler, tau 0.02, reward 1,
//    12-degree / 2.4 limits), reached through `env.step` at core.py:197.
//  * Hopper: a Hopper-v2-SHAPED surrogate (11-d obs, 3-d action, gear 200,
//    frame_skip 4, forward-velocity reward, Hopper-v2 health test).  MuJoCo is not
//    available, so its planar leg dynamics are a cost-representative stand-in.
#pragma once
#include "mrl_common.h"

#pragma clang fp contract(off)

namespace mrl {

// ------------------------------------------------------------------ CartPole-v0
constexpr int CP_NS = 4, CP_OBS = 4;
constexpr double CP_GRAVITY = 9.8, CP_MASSPOLE = 0.1, CP_TOTAL_MASS = 1.1, CP_LENGTH = 0.5;
constexpr double CP_POLEMASS_LENGTH = 0.05, CP_FORCE_MAG = 10.0, CP_TAU = 0.02;
constexpr double CP_THETA_THRESHOLD = 12 * 2 * 3.141592653589793 / 360;
constexpr double CP_X_THRESHOLD = 2.4;

__device__ inline void cartpole_reset(const double* u, double* s) {
  for (int i = 0; i < 4; ++i) s[i] = u[i] * 0.1 - 0.05;
}

__device__ inline void cartpole_step(double* s, int a, double& rew, bool& done) {
  const double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
  const double force = a == 1 ? CP_FORCE_MAG : -CP_FORCE_MAG;
  const double costheta = cos(theta);
  const double sintheta = sin(theta);
  const double temp = (force + CP_POLEMASS_LENGTH * theta_dot * theta_dot * sintheta) / CP_TOTAL_MASS;
  const double thetaacc = (CP_GRAVITY * sintheta - costheta * temp) /
                          (CP_LENGTH * (4.0 / 3.0 - CP_MASSPOLE * costheta * costheta / CP_TOTAL_MASS));
  const double xacc = temp - CP_POLEMASS_LENGTH * thetaacc * costheta / CP_TOTAL_MASS;
  const double nx = x + CP_TAU * x_dot;
  const double nxd = x_dot + CP_TAU * xacc;
  const double nt = theta + CP_TAU * theta_dot;
  const double ntd = theta_dot + CP_TAU * thetaacc;
  s[0] = nx; s[1] = nxd; s[2] = nt; s[3] = ntd;
  done = (nx < -CP_X_THRESHOLD) || (nx > CP_X_THRESHOLD) || (nt < -CP_THETA_THRESHOLD) || (nt > CP_THETA_THRESHOLD);
  rew = 1.0;
}

__device__ inline void cartpole_obs(const double* s, double* o) {
  for (int i = 0; i < 4; ++i) o[i] = s[i];
}

// ------------------------------------------------------------------ Hopper surrogate
constexpr int HP_NS = 12, HP_OBS = 11, HP_ACT = 3;
constexpr double HP_DT = 0.002;
constexpr int HP_FRAME_SKIP = 4;
constexpr double HP_GEAR = 200.0, HP_GRAV = 9.81, HP_MASS = 3.5, HP_I_ROOT = 2.0;
constexpr double HP_L_TORSO = 0.2, HP_L_THIGH = 0.45, HP_L_LEG = 0.5, HP_FOOT_R = 0.1;
constexpr double HP_KC = 5000.0, HP_CC = 60.0, HP_MU = 0.9, HP_VMAX = 50.0;

__device__ inline void hopper_reset(const double* u, double* s) {
  for (int i = 0; i < 6; ++i) s[i] = u[i] * 0.01 - 0.005;
  s[1] = s[1] + 1.25;
  for (int i = 0; i < 6; ++i) s[6 + i] = u[6 + i] * 0.01 - 0.005;
}

__device__ inline double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ inline void hopper_substep(double* q, double* v, const double* tau) {
  const double HP_I[3] = {4.0, 3.0, 1.5};
  const double HP_K[3] = {30.0, 30.0, 20.0};
  const double HP_C[3] = {8.0, 6.0, 4.0};
  const double x = q[0], z = q[1], ar = q[2], a1 = q[3], a2 = q[4], a3 = q[5];
  const double vx = v[0], vz = v[1], var_ = v[2], v1 = v[3], v2 = v[4], v3 = v[5];
  const double p1 = ar + a1;
  const double p2 = p1 + a2;
  const double w1 = var_ + v1;
  const double w2 = w1 + v2;
  double s0, c0, s1, c1, s2, c2;  // one shared range reduction per angle
  sincos(ar, &s0, &c0);
  sincos(p1, &s1, &c1);
  sincos(p2, &s2, &c2);
  const double fx = x + HP_L_TORSO * s0 + HP_L_THIGH * s1 + HP_L_LEG * s2;
  const double fz = z - HP_L_TORSO * c0 - HP_L_THIGH * c1 - HP_L_LEG * c2;
  const double fvx = vx + HP_L_TORSO * c0 * var_ + HP_L_THIGH * c1 * w1 + HP_L_LEG * c2 * w2;
  const double fvz = vz + HP_L_TORSO * s0 * var_ + HP_L_THIGH * s1 * w1 + HP_L_LEG * s2 * w2;
  const double pen = HP_FOOT_R - fz;
  const double fn = pen > 0.0 ? fmax(HP_KC * pen - HP_CC * fvz, 0.0) : 0.0;
  const double ft = -HP_MU * fn * tanh(fvx / 0.05) * (1.0 - 0.5 * fabs(sin(a3)));
  const double ax = ft / HP_MASS;
  const double az = fn / HP_MASS - HP_GRAV;
  const double tq_root = (fx - x) * fn - (fz - z) * ft;
  const double hx = x + HP_L_TORSO * s0;
  const double hz = z - HP_L_TORSO * c0;
  const double kx = hx + HP_L_THIGH * s1;
  const double kz = hz - HP_L_THIGH * c1;
  const double tq1 = (fx - hx) * fn - (fz - hz) * ft;
  const double tq2 = (fx - kx) * fn - (fz - kz) * ft;
  double acc[6];
  acc[0] = ax;
  acc[1] = az;
  acc[2] = (0.05 * tq_root - tau[0] * 0.1 - 1.0 * var_) / HP_I_ROOT;
  acc[3] = (tau[0] - HP_K[0] * a1 - HP_C[0] * v1 + 0.05 * tq1) / HP_I[0];
  acc[4] = (tau[1] - HP_K[1] * a2 - HP_C[1] * v2 + 0.05 * tq2) / HP_I[1];
  acc[5] = (tau[2] - HP_K[2] * a3 - HP_C[2] * v3 - 0.02 * ft) / HP_I[2];
  for (int i = 0; i < 6; ++i) v[i] = clampd(v[i] + HP_DT * acc[i], -HP_VMAX, HP_VMAX);
  for (int i = 0; i < 6; ++i) q[i] = q[i] + HP_DT * v[i];
  const double lo[3] = {-2.61799, -2.61799, -0.785398};
  const double hi[3] = {0.0, 0.0, 0.785398};
  for (int jj = 0; jj < 3; ++jj) {
    const int j = 3 + jj;
    const bool over = q[j] > hi[jj];
    const bool under = q[j] < lo[jj];
    q[j] = over ? hi[jj] : (under ? lo[jj] : q[j]);
    if (over || under) v[j] = 0.0;
  }
}

__device__ inline void hopper_step(double* s, const float* a, double& rew, bool& done) {
  double tau[3];
  double asq = 0.0;
  for (int j = 0; j < 3; ++j) {
    const double aj = (double)a[j];
    tau[j] = HP_GEAR * clampd(aj, -1.0, 1.0);
    asq += aj * aj;
  }
  double* q = s;
  double* v = s + 6;
  const double x_before = q[0];
  for (int k = 0; k < HP_FRAME_SKIP; ++k) hopper_substep(q, v, tau);
  rew = (q[0] - x_before) / (HP_DT * HP_FRAME_SKIP) + 1.0 - 1e-3 * asq;
  bool healthy = true;
  for (int i = 0; i < 12; ++i) healthy = healthy && isfinite(s[i]);
  for (int i = 2; i < 12; ++i) healthy = healthy && (fabs(s[i]) < 100.0);
  healthy = healthy && (q[1] > 0.7) && (fabs(q[2]) < 0.2);
  done = !healthy;
}

__device__ inline void hopper_obs(const double* s, double* o) {
  for (int i = 0; i < 5; ++i) o[i] = s[1 + i];
  for (int i = 0; i < 6; ++i) o[5 + i] = clampd(s[6 + i], -10.0, 10.0);
}

}  // namespace mrl
