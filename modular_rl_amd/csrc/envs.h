// Batched env dynamics on device (fp64, struct-of-arrays state), operation-for-
// operation twins of oracle/envs.py.  FMA contraction is disabled so the results
// follow the same rounding sequence as the numpy oracle.
//
//  * CartPole-v0: gym's classic-control equations (Euler, tau 0.02, reward 1,
//    12-degree / 2.4 limits), reached through `env.step` at core.py:197.
//  * Humanoid: a Humanoid-v2-SHAPED surrogate (376-d obs, 17-d action in [-.4, .4],
//    frame_skip 5 x dt 0.003, 1.25 v + 5 alive - 0.1|a|^2 - impact, 1 < z < 2), a
//    sagittal two-leg contact model with 17 damped actuated joints (oracle/envs.py).
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

// the four angle functions of a substep: (s0,c0)=sincos(ar), (s1,c1)=sincos(p1),
// (s2,c2)=sincos(p2), sa3=sin(a3); one shared range reduction per angle
struct HopperTrigSerial {
  __device__ void operator()(double ar, double p1, double p2, double a3, double* sc) const {
    sincos(ar, &sc[0], &sc[1]);
    sincos(p1, &sc[2], &sc[3]);
    sincos(p2, &sc[4], &sc[5]);
    sc[6] = sin(a3);
  }
};

template <class Trig>
__device__ inline void hopper_substep(double* q, double* v, const double* tau, const Trig& trig) {
  const double HP_I[3] = {4.0, 3.0, 1.5};
  const double HP_K[3] = {30.0, 30.0, 20.0};
  const double HP_C[3] = {8.0, 6.0, 4.0};
  const double x = q[0], z = q[1], ar = q[2], a1 = q[3], a2 = q[4], a3 = q[5];
  const double vx = v[0], vz = v[1], var_ = v[2], v1 = v[3], v2 = v[4], v3 = v[5];
  const double p1 = ar + a1;
  const double p2 = p1 + a2;
  const double w1 = var_ + v1;
  const double w2 = w1 + v2;
  double sc[7];
  trig(ar, p1, p2, a3, sc);
  const double s0 = sc[0], c0 = sc[1], s1 = sc[2], c1 = sc[3], s2 = sc[4], c2 = sc[5];
  const double fx = x + HP_L_TORSO * s0 + HP_L_THIGH * s1 + HP_L_LEG * s2;
  const double fz = z - HP_L_TORSO * c0 - HP_L_THIGH * c1 - HP_L_LEG * c2;
  const double fvx = vx + HP_L_TORSO * c0 * var_ + HP_L_THIGH * c1 * w1 + HP_L_LEG * c2 * w2;
  const double fvz = vz + HP_L_TORSO * s0 * var_ + HP_L_THIGH * s1 * w1 + HP_L_LEG * s2 * w2;
  const double pen = HP_FOOT_R - fz;
  const double fn = pen > 0.0 ? fmax(HP_KC * pen - HP_CC * fvz, 0.0) : 0.0;
  const double ft = -HP_MU * fn * tanh(fvx / 0.05) * (1.0 - 0.5 * fabs(sc[6]));
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

template <class Trig = HopperTrigSerial>
__device__ inline void hopper_step(double* s, const float* a, double& rew, bool& done, const Trig& trig = Trig()) {
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
  for (int k = 0; k < HP_FRAME_SKIP; ++k) hopper_substep(q, v, tau, trig);
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

// ------------------------------------------------------------------ Humanoid surrogate
// state: q[23] (x, y, z, roll, pitch, yaw, 17 joints) ++ v[23] ++ last torques[17]
constexpr int HM_NQ = 23, HM_NV = 23, HM_ACT = 17, HM_NS = 63, HM_OBS = 376, HM_NU = 46;
constexpr double HM_DT = 0.003;
constexpr int HM_FRAME_SKIP = 5;
constexpr double HM_GEAR = 100.0, HM_ACT_LIM = 0.4, HM_MASS = 40.0, HM_GRAV = 9.81;
constexpr double HM_L_THIGH = 0.42, HM_L_SHIN = 0.42, HM_HIP_DROP = 0.5, HM_FOOT_R = 0.05;
constexpr double HM_KC = 20000.0, HM_CC = 800.0, HM_MU = 0.9, HM_VMAX = 50.0;
constexpr double HM_I_ROOT0 = 8.0, HM_I_ROOT1 = 6.0, HM_I_ROOT2 = 6.0;
constexpr double HM_K_ROOT0 = 20.0, HM_K_ROOT1 = 5.0, HM_TOPPLE = 120.0;
constexpr double HM_C_ROOT0 = 30.0, HM_C_ROOT1 = 30.0, HM_C_ROOT2 = 10.0;
constexpr double HM_I_J = 1.0, HM_K_J = 100.0, HM_C_J = 10.0, HM_Z0 = 1.4;

__device__ inline double hm_body_mass(int b) {
  constexpr double m[14] = {8.0, 2.0, 6.0, 4.5, 2.6, 1.2, 4.5, 2.6, 1.2, 1.6, 1.2, 1.6, 1.2, 2.0};
  return m[b];
}
__device__ inline void hm_limits(int j, double& lo, double& hi) {
  if (j == 6 || j == 10) { lo = -2.5; hi = 0.0; }
  else if (j == 13 || j == 16) { lo = -2.0; hi = 0.5; }
  else { lo = -1.0; hi = 1.0; }
}

__device__ inline void humanoid_reset(const double* u, double* s) {
  for (int i = 0; i < HM_NQ; ++i) s[i] = u[i] * 0.02 - 0.01;
  s[2] = s[2] + HM_Z0;
  for (int i = 0; i < HM_NV; ++i) s[HM_NQ + i] = u[HM_NQ + i] * 0.02 - 0.01;
  for (int i = 0; i < HM_ACT; ++i) s[HM_NQ + HM_NV + i] = 0.0;
}

// foot of one leg (hip_y joint hy, knee kn): position x/z, normal and friction force
__device__ inline void hm_leg(const double* q, const double* v, int hy, int kn, double& fx, double& fz, double& fn,
                              double& ft) {
  const double a1 = q[4] + q[6 + hy];
  const double a2 = a1 + q[6 + kn];
  const double w1 = v[4] + v[6 + hy];
  const double w2 = w1 + v[6 + kn];
  double s1, c1, s2, c2;
  sincos(a1, &s1, &c1);
  sincos(a2, &s2, &c2);
  fx = (q[0] + HM_L_THIGH * s1) + HM_L_SHIN * s2;
  fz = ((q[2] - HM_HIP_DROP) - HM_L_THIGH * c1) - HM_L_SHIN * c2;
  const double fvx = (v[0] + (HM_L_THIGH * c1) * w1) + (HM_L_SHIN * c2) * w2;
  const double fvz = (v[2] + (HM_L_THIGH * s1) * w1) + (HM_L_SHIN * s2) * w2;
  const double pen = HM_FOOT_R - fz;
  fn = pen > 0.0 ? fmax(HM_KC * pen - HM_CC * fvz, 0.0) : 0.0;
  ft = (-HM_MU * fn) * tanh(fvx / 0.05);
}

__device__ inline void humanoid_substep(double* q, double* v, const double* tau) {
  double fxr, fzr, fnr, ftr, fxl, fzl, fnl, ftl;
  hm_leg(q, v, 5, 6, fxr, fzr, fnr, ftr);
  hm_leg(q, v, 9, 10, fxl, fzl, fnl, ftl);
  const double x = q[0], z = q[2];
  double acc[HM_NV];
  acc[0] = (ftr + ftl) / HM_MASS;
  acc[1] = -0.5 * v[1];
  acc[2] = (fnr + fnl) / HM_MASS - HM_GRAV;
  const double tq_p = ((fxr - x) * fnr - (fzr - z) * ftr) + ((fxl - x) * fnl - (fzl - z) * ftl);
  acc[3] = ((((HM_TOPPLE * sin(q[3]) - HM_K_ROOT0 * q[3]) - HM_C_ROOT0 * v[3]) + 0.02 * (tau[3] - tau[7])) +
            0.01 * (fnr - fnl)) / HM_I_ROOT0;
  acc[4] = ((((HM_TOPPLE * sin(q[4]) + 0.02 * tq_p) - HM_K_ROOT1 * q[4]) - HM_C_ROOT1 * v[4]) -
            0.05 * (tau[5] + tau[9])) / HM_I_ROOT1;
  acc[5] = (0.02 * (tau[4] + tau[8]) - HM_C_ROOT2 * v[5]) / HM_I_ROOT2;
#pragma unroll
  for (int j = 0; j < HM_ACT; ++j) {
    const double qj = q[6 + j], vj = v[6 + j];
    double a = (tau[j] - HM_K_J * qj) - HM_C_J * vj;
    if (j >= 3 && j <= 6) a = a + (0.03 * fnr) * sin(qj);
    else if (j >= 7 && j <= 10) a = a + (0.03 * fnl) * sin(qj);
    acc[6 + j] = a / HM_I_J;
  }
#pragma unroll
  for (int i = 0; i < HM_NV; ++i) v[i] = clampd(v[i] + HM_DT * acc[i], -HM_VMAX, HM_VMAX);
#pragma unroll
  for (int i = 0; i < HM_NQ; ++i) q[i] = q[i] + HM_DT * v[i];
#pragma unroll
  for (int j = 0; j < HM_ACT; ++j) {
    double lo, hi;
    hm_limits(j, lo, hi);
    const bool over = q[6 + j] > hi;
    const bool under = q[6 + j] < lo;
    q[6 + j] = over ? hi : (under ? lo : q[6 + j]);
    if (over || under) v[6 + j] = 0.0;
  }
}

__device__ inline void humanoid_step(double* s, const float* a, double& rew, bool& done) {
  double* q = s;
  double* v = s + HM_NQ;
  double* tau = s + HM_NQ + HM_NV;
  double asq = 0.0;
#pragma unroll
  for (int j = 0; j < HM_ACT; ++j) {
    const double aj = (double)a[j];
    tau[j] = HM_GEAR * clampd(aj, -HM_ACT_LIM, HM_ACT_LIM);
    asq = asq + aj * aj;
  }
  const double x_before = q[0];
  for (int k = 0; k < HM_FRAME_SKIP; ++k) humanoid_substep(q, v, tau);
  double fxr, fzr, fnr, ftr, fxl, fzl, fnl, ftl;
  hm_leg(q, v, 5, 6, fxr, fzr, fnr, ftr);
  hm_leg(q, v, 9, 10, fxl, fzl, fnl, ftl);
  const double cfrc = ((fnr * fnr + ftr * ftr) + fnl * fnl) + ftl * ftl;
  const double impact = fmin(5e-7 * cfrc, 10.0);
  rew = ((1.25 * (q[0] - x_before) / (HM_DT * HM_FRAME_SKIP) + 5.0) - 0.1 * asq) - impact;
  bool healthy = true;
#pragma unroll
  for (int i = 0; i < HM_NS; ++i) healthy = healthy && isfinite(s[i]);
  healthy = healthy && (q[2] > 1.0) && (q[2] < 2.0);
  done = !healthy;
}

// 376-d observation, written through out(k, value) (SoA global rows on the layered path)
template <class Out>
__device__ inline void humanoid_obs(const double* s, Out out) {
  const double* q = s;
  const double* v = s + HM_NQ;
  const double* tau = s + HM_NQ + HM_NV;
#pragma unroll
  for (int i = 0; i < 21; ++i) out(i, q[2 + i]);
  out(21, cos(q[4]));
#pragma unroll
  for (int i = 0; i < HM_NV; ++i) out(22 + i, v[i]);
#pragma unroll
  for (int b = 0; b < 14; ++b) {
    const double phi = q[6 + b];
    const double m = hm_body_mass(b);
    const int base = 45 + 10 * b;
    for (int k = 0; k < 5; ++k) out(base + k, m * cos((double)k * phi));
    for (int k = 1; k < 6; ++k) out(base + 4 + k, m * sin((double)k * phi));
    double sph, cph;
    sincos(phi, &sph, &cph);
    const int cb = 185 + 6 * b;
    out(cb + 0, v[6 + b]);
    out(cb + 1, v[3 + b % 3]);
    out(cb + 2, v[0] * cph);
    out(cb + 3, v[2] * sph);
    out(cb + 4, v[6 + b] * cph);
    out(cb + 5, v[6 + b] * sph);
  }
  for (int i = 0; i < 6; ++i) out(269 + i, 0.0);
#pragma unroll
  for (int i = 0; i < HM_ACT; ++i) out(275 + i, tau[i]);
  double fxr, fzr, fnr, ftr, fxl, fzl, fnl, ftl;
  hm_leg(q, v, 5, 6, fxr, fzr, fnr, ftr);
  hm_leg(q, v, 9, 10, fxl, fzl, fnl, ftl);
  for (int i = 0; i < 84; ++i) {
    double val = 0.0;
    if (i == 36) val = fnr;
    else if (i == 37) val = ftr;
    else if (i == 54) val = fnl;
    else if (i == 55) val = ftl;
    out(292 + i, val);
  }
}

}  // namespace mrl
