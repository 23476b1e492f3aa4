// Batched env dynamics on device (fp64, struct-of-arrays state), operation-for-
// operation twins of oracle/envs.py.  FMA contraction is disabled so the results
// follow the same rounding sequence as the numpy oracle; the Hopper step fuses
// multiply-adds only at explicit fmad() calls, which the oracle mirrors exactly
// (oracle/fma.py).
//
//  * CartPole-v0: gym's classic-control equations (Euler, tau 0.02, reward 1,
//    12-degree / 2.4 limits), reached through `env.step` at core.py:197.
//  * Humanoid-v2: gym's humanoid.xml as 3-D articulated rigid-body dynamics
//    (humanoid.h, twin of oracle/humanoid.py).
//  * Hopper-v2: gym's hopper.xml as planar articulated rigid-body dynamics with
//    compliant ground contact (11-d obs, 3-d action, gear 200, frame_skip 4,
//    forward-velocity reward, Hopper-v2 health test); MuJoCo itself is absent.
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

// ------------------------------------------------------------------ Hopper-v2
// gym's hopper.xml as planar articulated rigid-body dynamics (oracle/envs.py has
// the model, its constants and this exact operation order):
// q = (rootx, rootz, rooty, thigh, leg, foot),  M(q) qdd = tau - h(q, qd) + J_c^T f_c.
// One dt: pivot kinematics root -> foot; compliant ground contact at the two
// end-spheres of each capsule; subtree force / moment sums (RNEA: tau_c - h) and
// composite inertias (CRBA: M) foot -> root; the translational block
// (M_tt = total mass * I) eliminated by its Schur complement; a 4x4 LDL^T solve;
// semi-implicit Euler.  frame_skip 4 x dt 0.002.  The fused step kernel splits
// the contact work and the angle functions over the four 16-lane rows that hold
// the same envs (HopperQuad, rollout.hip); everything else is evaluated by every
// row in the same order, so all rows continue with the identical state.
constexpr int HP_NS = 12, HP_OBS = 11, HP_ACT = 3;
constexpr double HP_DT = 0.002;
constexpr int HP_FRAME_SKIP = 4;
constexpr double HP_GEAR = 200.0, HP_GRAV = 9.81;
constexpr double HP_KC = 20000.0, HP_CC = 400.0, HP_CF = 1000.0;
constexpr double HP_DAMP = 1.0, HP_ARM = 1.0, HP_KL = 2000.0, HP_CL = 50.0;
constexpr double HP_MASS[4] = {3.6651914291880923, 4.057890510886817, 2.7813566959781637, 5.315574769873929};
constexpr double HP_INERTIA[4] = {0.06924593807287505, 0.0932987568269219, 0.07230254017320971,
                                  0.10352308059000535};
constexpr double HP_SEG[3] = {0.2, 0.45, 0.5};
constexpr double HP_COMX[4] = {0.0, 0.0, 0.0, 0.065}, HP_COMZ[4] = {0.0, -0.225, -0.25, 0.0};
constexpr double HP_MB3 = HP_MASS[3], HP_MB2 = HP_MASS[2] + HP_MB3, HP_MB1 = HP_MASS[1] + HP_MB2,
                 HP_MB0 = HP_MASS[0] + HP_MB1;  // subtree masses
constexpr double HP_MB[4] = {HP_MB0, HP_MB1, HP_MB2, HP_MB3};
constexpr double HP_IMT = 1.0 / HP_MB0;

// a0..a3 by k.  With k a run-time lane value (HopperQuad: the lane's row) the select
// tree is formed from bit masks the optimiser cannot see through: a plain ternary chain
// on doubles was compiled into a switch on k -- exec-masked branches around every
// selection, all four arms issued by the divergent rows, about a dozen times per
// substep.  Exact either way (a selection).
__device__ inline double pick_bits(uint32_t m, double x, double y) {  // m ? y : x, m all ones or zero
  const uint64_t xb = (uint64_t)__double_as_longlong(x), yb = (uint64_t)__double_as_longlong(y);
  const uint32_t lo = ((uint32_t)yb & m) | ((uint32_t)xb & ~m);
  const uint32_t hi = ((uint32_t)(yb >> 32) & m) | ((uint32_t)(xb >> 32) & ~m);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
#ifndef MRL_HP_SEL_BITS  // 0: the plain ternary chain (A/B: r04x rollout 13.87 ms with, 14.05 without);
#define MRL_HP_SEL_BITS 2  // 1: bit masks made opaque per call; 2: selects on k's bits
#endif
#ifndef MRL_HP_LIM_BITS  // 1: joint limits and the health test without branches as well (measured
#define MRL_HP_LIM_BITS 0  // slower: 14.56 ms, the extra live values spill)
#endif
#ifndef MRL_HP_LIM_SEL  // 1: joint limits as selects over both evaluated forms (0: the ternary)
#define MRL_HP_LIM_SEL 1
#endif
#ifndef MRL_HP_HEALTH_BITS  // 1: the health test's comparisons combined with & (no branches)
#define MRL_HP_HEALTH_BITS 1
#endif
__device__ inline double sel4(int k, double a0, double a1, double a2, double a3) {
  if (!MRL_HP_SEL_BITS || __builtin_constant_p(k)) return k == 0 ? a0 : (k == 1 ? a1 : (k == 2 ? a2 : a3));
  if (MRL_HP_SEL_BITS == 2) {  // selects on k's two bits (v_cndmask on loop-invariant lane masks)
    const bool b0 = (k & 1) != 0, b1 = (k & 2) != 0;
    const double lo = b0 ? a1 : a0, hi = b0 ? a3 : a2;
    return b1 ? hi : lo;
  }
  uint32_t m0 = 0u - (uint32_t)(k & 1), m1 = 0u - (uint32_t)((k >> 1) & 1);
  asm volatile("" : "+v"(m0), "+v"(m1));
  return pick_bits(m1, pick_bits(m0, a0, a1), pick_bits(m0, a2, a3));
}

__device__ inline void hopper_reset(const double* u, double* s) {
  for (int i = 0; i < 6; ++i) s[i] = u[i] * 0.01 - 0.005;
  s[1] = s[1] + 1.25;
  for (int i = 0; i < 6; ++i) s[6 + i] = u[6 + i] * 0.01 - 0.005;
}

__device__ inline double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

// a * b + c with one rounding (v_fma_f64).  FMA contraction stays off in this file, so
// only these explicit calls fuse, at the places the oracle fuses with its exact
// emulation (oracle/fma.py) -- the GPU and numpy dynamics stay bit-identical.
__device__ inline double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

// capsule k's contact constants: radius, friction, the two end-spheres' offsets (u, w)
// in the segment frame -- [field][k] in HP_CAP (the fused rollout keeps this table in LDS:
// its lanes' k is their row, so a select per constant per substep became one LDS read)
struct CapsuleC {
  double rad, mu, u0, u1, w0, w1;
};
constexpr double HP_CAP[24] = {0.05, 0.05, 0.04, 0.06,  1.0, 1.0, 1.0, 2.0,  0.0, 0.0, 0.0, -0.13,
                               0.0, 0.0, 0.0, 0.26,      0.2, 0.0, 0.0, 0.0,  -0.2, -0.45, -0.5, 0.0};
__device__ inline CapsuleC capsule_const(int k) {
  return CapsuleC{sel4(k, HP_CAP[0], HP_CAP[1], HP_CAP[2], HP_CAP[3]),
                  sel4(k, HP_CAP[4], HP_CAP[5], HP_CAP[6], HP_CAP[7]),
                  sel4(k, HP_CAP[8], HP_CAP[9], HP_CAP[10], HP_CAP[11]),
                  sel4(k, HP_CAP[12], HP_CAP[13], HP_CAP[14], HP_CAP[15]),
                  sel4(k, HP_CAP[16], HP_CAP[17], HP_CAP[18], HP_CAP[19]),
                  sel4(k, HP_CAP[20], HP_CAP[21], HP_CAP[22], HP_CAP[23])};
}

// capsule k's two end-spheres against the floor: contact force sum (x, z) and
// moment about pivot k (oracle hopper_contacts); cc = capsule k's constants
__device__ inline void hopper_contacts(const CapsuleC& cc, double pz, double pvx, double pvz, double om, double sk,
                                       double ck, double* out) {
  const double rad = cc.rad, mu = cc.mu;
  double fcx = 0.0, fcz = 0.0, ncm = 0.0;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const double u = n == 0 ? cc.u0 : cc.u1;
    const double w = n == 0 ? cc.w0 : cc.w1;
    const double ox = fmad(u, ck, w * sk);
    const double oz = fmad(w, ck, -(u * sk)) - rad;
    const double pen = -(pz + oz);
    const double vx = fmad(om, oz, pvx);
    const double vz = fmad(-om, ox, pvz);
    const double fnr = fmad(HP_KC, pen, -(HP_CC * vz));
    const double fn = pen > 0.0 ? (fnr > 0.0 ? fnr : 0.0) : 0.0;
    const double lim = mu * fn;
    const double fv = HP_CF * vx;
    const double fl = fv > -lim ? fv : -lim;
    const double ft = -(fl < lim ? fl : lim);
    fcx = fcx + ft;
    fcz = fcz + fn;
    ncm = ncm + fmad(oz, ft, -(ox * fn));
  }
  out[0] = fcx;
  out[1] = fcz;
  out[2] = ncm;
}

// every lane evaluates the whole env (layered rollout)
struct HopperSerial {
  __device__ CapsuleC capsule(int k) const { return capsule_const(k); }
  __device__ void sincos4(const double* phi, double* s, double* c, double&, double&) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) sincos(phi[k], &s[k], &c[k]);
  }
  // segment k's value of a per-segment array (k a compile-time index here)
  __device__ double own(int k, const double* a4, double) const { return a4[k]; }
  template <class F>
  __device__ void contacts(F f, double (*ct)[3]) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) f(k, ct[k]);
  }
};

// LDL^T solve of the 4x4 SPD system K x = r (oracle hopper_ldl4)
__device__ inline void ldl_solve4(const double (&K)[4][4], const double* r, double* x) {
  double L[4][4], D[4], iD[4], y[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double d = K[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d = fmad(-(L[j][k] * L[j][k]), D[k], d);
    D[j] = d;
    iD[j] = 1.0 / d;
#pragma unroll
    for (int i = j + 1; i < 4; ++i) {
      double acc = K[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) acc = fmad(-(L[i][k] * L[j][k]), D[k], acc);
      L[i][j] = acc * iD[j];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double acc = r[i];
#pragma unroll
    for (int k = 0; k < i; ++k) acc = fmad(-L[i][k], y[k], acc);
    y[i] = acc;
  }
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    double acc = y[i] * iD[i];
#pragma unroll
    for (int k = i + 1; k < 4; ++k) acc = fmad(-L[k][i], x[k], acc);
    x[i] = acc;
  }
}

template <class Par>
__device__ inline void hopper_substep(double* q, double* v, const double* tau, const Par& par) {
  const double HP_LO[3] = {-2.6179938779914944, -2.6179938779914944, -0.7853981633974483};
  const double HP_HI[3] = {0.0, 0.0, 0.7853981633974483};
  double phi[4], sg[4], cg[4], om[4];
  phi[0] = q[2];
#pragma unroll
  for (int j = 1; j < 4; ++j) phi[j] = phi[j - 1] - q[2 + j];
#ifdef MRL_HP_ABL_NOSINCOS  // diagnostic timing build only (results are wrong)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sg[k] = phi[k] - phi[k] * phi[k] * phi[k] * (1.0 / 6.0);
    cg[k] = 1.0 - phi[k] * phi[k] * 0.5;
  }
#else
  double s_own = 0.0, c_own = 0.0;  // HopperQuad: the row's own segment's sin / cos
  par.sincos4(phi, sg, cg, s_own, c_own);
#endif
  om[0] = v[2];
#pragma unroll
  for (int j = 1; j < 4; ++j) om[j] = om[j - 1] - v[2 + j];
  double gx[3], gz[3], rx[4], rz[4];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    gx[j] = -HP_SEG[j] * sg[j];
    gz[j] = -HP_SEG[j] * cg[j];
  }
  // COM offsets: (0, COMZ) on the torso / thigh / leg, (COMX, 0) on the foot
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    rx[k] = HP_COMZ[k] * sg[k];
    rz[k] = HP_COMZ[k] * cg[k];
  }
  rx[3] = HP_COMX[3] * cg[3];
  rz[3] = -(HP_COMX[3] * sg[3]);
  // pivots: height, velocity, bias acceleration (root -> foot)
  double pz[4], pvx[4], pvz[4], pax[4], paz[4];
  pz[0] = q[1];
  pvx[0] = v[0];
  pvz[0] = v[1];
  pax[0] = 0.0;
  paz[0] = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double w2 = om[j] * om[j];
    pz[j + 1] = pz[j] + gz[j];
    pvx[j + 1] = fmad(om[j], gz[j], pvx[j]);
    pvz[j + 1] = fmad(-om[j], gx[j], pvz[j]);
    pax[j + 1] = fmad(-w2, gx[j], pax[j]);
    paz[j + 1] = fmad(-w2, gz[j], paz[j]);
  }
  double ct[4][3];
#ifdef MRL_HP_ABL_NOCONTACT  // diagnostic timing build only (results are wrong)
#pragma unroll
  for (int k = 0; k < 4; ++k) ct[k][0] = ct[k][1] = ct[k][2] = pz[k] * 1e-3;
  if (false)
#endif
  par.contacts(
      [&](int k, double* out) {
        hopper_contacts(par.capsule(k), sel4(k, pz[0], pz[1], pz[2], pz[3]), sel4(k, pvx[0], pvx[1], pvx[2], pvx[3]),
                        sel4(k, pvz[0], pvz[1], pvz[2], pvz[3]), sel4(k, om[0], om[1], om[2], om[3]),
                        par.own(k, sg, s_own), par.own(k, cg, c_own), out);
      },
      ct);
  // per body: inertial + gravity force minus contact force, moment about its pivot
  double Fx[4], Fz[4], N[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double w2 = om[k] * om[k];
    const double mx = HP_MASS[k] * fmad(-w2, rx[k], pax[k]);
    const double mz = HP_MASS[k] * (fmad(-w2, rz[k], paz[k]) + HP_GRAV);
    Fx[k] = mx - ct[k][0];
    Fz[k] = mz - ct[k][1];
    N[k] = fmad(rz[k], mx, -(rx[k] * mz)) - ct[k][2];
  }
  // subtree sums about pivot k (foot -> root)
  double Fbx[4], Fbz[4], Nb[4], Sx[4], Sz[4], J[4];
  Fbx[3] = Fx[3];
  Fbz[3] = Fz[3];
  Nb[3] = N[3];
  Sx[3] = HP_MASS[3] * rx[3];
  Sz[3] = HP_MASS[3] * rz[3];
  J[3] = fmad(HP_MASS[3], fmad(rx[3], rx[3], rz[3] * rz[3]), HP_INERTIA[3]);
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    Nb[k] = (N[k] + Nb[k + 1]) + fmad(gz[k], Fbx[k + 1], -(gx[k] * Fbz[k + 1]));
    Fbx[k] = Fx[k] + Fbx[k + 1];
    Fbz[k] = Fz[k] + Fbz[k + 1];
    J[k] = (fmad(HP_MASS[k], fmad(rx[k], rx[k], rz[k] * rz[k]), HP_INERTIA[k]) + J[k + 1]) +
           fmad(2.0, fmad(gx[k], Sx[k + 1], gz[k] * Sz[k + 1]), HP_MB[k + 1] * (HP_SEG[k] * HP_SEG[k]));
    Sx[k] = fmad(HP_MB[k + 1], gx[k], fmad(HP_MASS[k], rx[k], Sx[k + 1]));
    Sz[k] = fmad(HP_MB[k + 1], gz[k], fmad(HP_MASS[k], rz[k], Sz[k + 1]));
  }
  double rhs[6] = {-Fbx[0], -Fbz[0], -Nb[0], Nb[1], Nb[2], Nb[3]};
  // rotational block C and coupling rows B0 / B1 of M (oracle hopper_dynamics_terms)
  double Dx[4][4], Dz[4][4];
  Dx[0][1] = gx[0];
  Dz[0][1] = gz[0];
  Dx[1][2] = gx[1];
  Dz[1][2] = gz[1];
  Dx[2][3] = gx[2];
  Dz[2][3] = gz[2];
  Dx[0][2] = gx[0] + gx[1];
  Dz[0][2] = gz[0] + gz[1];
  Dx[0][3] = Dx[0][2] + gx[2];
  Dz[0][3] = Dz[0][2] + gz[2];
  Dx[1][3] = gx[1] + gx[2];
  Dz[1][3] = gz[1] + gz[2];
  double C[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    C[a][a] = J[a];
#pragma unroll
    for (int b = a + 1; b < 4; ++b) {
      const double val = fmad(Dx[a][b], Sx[b], fmad(Dz[a][b], Sz[b], J[b]));
      C[a][b] = a == 0 ? -val : val;
    }
  }
  const double B0[4] = {Sz[0], -Sz[1], -Sz[2], -Sz[3]};
  const double B1[4] = {-Sx[0], Sx[1], Sx[2], Sx[3]};
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const int jj = i - 1, j = 2 + i;
    C[i][i] = C[i][i] + HP_ARM;
#if MRL_HP_LIM_SEL
    // joint-limit force: both one-sided forms evaluated, the active one picked by a plain
    // select (v_cndmask) -- the ternary over the fmas was an exec-masked branch pair per
    // joint, both arms issued by divergent rows
    const double cv = -(HP_CL * v[j]);
    const double flo = fmad(HP_KL, HP_LO[jj] - q[j], cv), fhi = fmad(HP_KL, HP_HI[jj] - q[j], cv);
    const double lim = q[j] < HP_LO[jj] ? flo : (q[j] > HP_HI[jj] ? fhi : 0.0);
#elif MRL_HP_LIM_BITS
    // joint-limit force: both one-sided forms evaluated, the active one selected by bit
    // masks (divergent rows make the ternary an exec-masked branch pair per joint)
    const double cv = -(HP_CL * v[j]);
    const double flo = fmad(HP_KL, HP_LO[jj] - q[j], cv), fhi = fmad(HP_KL, HP_HI[jj] - q[j], cv);
    uint32_t mlo = q[j] < HP_LO[jj] ? ~0u : 0u, mhi = q[j] > HP_HI[jj] ? ~0u : 0u;
    asm volatile("" : "+v"(mlo), "+v"(mhi));
    const double lim = pick_bits(mlo, pick_bits(mhi, 0.0, fhi), flo);
#else
    const double lim = q[j] < HP_LO[jj] ? fmad(HP_KL, HP_LO[jj] - q[j], -(HP_CL * v[j]))
                                        : (q[j] > HP_HI[jj] ? fmad(HP_KL, HP_HI[jj] - q[j], -(HP_CL * v[j])) : 0.0);
#endif
    rhs[j] = fmad(-HP_DAMP, v[j], rhs[j] + tau[jj]) + lim;
  }
  // Schur complement of the translational block, 4x4 LDL^T (oracle hopper_solve)
  double K[4][4], rr[4], x[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = a; b < 4; ++b) {
      K[a][b] = fmad(-fmad(B0[a], B0[b], B1[a] * B1[b]), HP_IMT, C[a][b]);
      K[b][a] = K[a][b];
    }
#pragma unroll
  for (int a = 0; a < 4; ++a) rr[a] = fmad(-fmad(B0[a], rhs[0], B1[a] * rhs[1]), HP_IMT, rhs[2 + a]);
#ifdef MRL_HP_ABL_NOLDL  // diagnostic timing build only (results are wrong)
#pragma unroll
  for (int a = 0; a < 4; ++a) x[a] = rr[a] * K[a][a];
#else
  ldl_solve4(K, rr, x);
#endif
  const double t0 = rhs[0] - fmad(B0[3], x[3], fmad(B0[2], x[2], fmad(B0[1], x[1], B0[0] * x[0])));
  const double t1 = rhs[1] - fmad(B1[3], x[3], fmad(B1[2], x[2], fmad(B1[1], x[1], B1[0] * x[0])));
  const double qdd[6] = {t0 * HP_IMT, t1 * HP_IMT, x[0], x[1], x[2], x[3]};
#pragma unroll
  for (int i = 0; i < 6; ++i) v[i] = fmad(HP_DT, qdd[i], v[i]);
#pragma unroll
  for (int i = 0; i < 6; ++i) q[i] = fmad(HP_DT, v[i], q[i]);
}

template <class Par = HopperSerial>
__device__ inline void hopper_step(double* s, const float* a, double& rew, bool& done, const Par& par = Par()) {
  double tau[3];
  for (int j = 0; j < 3; ++j) tau[j] = HP_GEAR * clampd((double)a[j], -1.0, 1.0);
  const double a0 = (double)a[0], a1 = (double)a[1], a2 = (double)a[2];
  const double asq = ((a0 * a0) + (a1 * a1)) + (a2 * a2);
  double* q = s;
  double* v = s + 6;
  const double x_before = q[0];
  for (int k = 0; k < HP_FRAME_SKIP; ++k) hopper_substep(q, v, tau, par);
  rew = (q[0] - x_before) / (HP_DT * HP_FRAME_SKIP) + 1.0 - 1e-3 * asq;
  bool healthy = true;
#if MRL_HP_LIM_BITS || MRL_HP_HEALTH_BITS  // every test evaluated and combined with & (the && chain: nested branches)
  // |s_i| < 100 is false for a NaN or an infinity, so isfinite(s_i) adds nothing for
  // i >= 2: the same truth value from 14 comparisons instead of 24, combined as a
  // balanced tree (depth 4) instead of a chain
  bool t[14];
  t[0] = isfinite(s[0]);
  t[1] = isfinite(s[1]);
#pragma unroll
  for (int i = 2; i < 12; ++i) t[i] = fabs(s[i]) < 100.0;
  t[12] = q[1] > 0.7;
  t[13] = fabs(q[2]) < 0.2;
#pragma unroll
  for (int w = 1; w < 14; w *= 2)
#pragma unroll
    for (int i = 0; i + w < 14; i += 2 * w) t[i] = t[i] & t[i + w];
  healthy = t[0];
#else
  for (int i = 0; i < 12; ++i) healthy = healthy && isfinite(s[i]);
  for (int i = 2; i < 12; ++i) healthy = healthy && (fabs(s[i]) < 100.0);
  healthy = healthy && (q[1] > 0.7) && (fabs(q[2]) < 0.2);
#endif
  done = !healthy;
}

__device__ inline void hopper_obs(const double* s, double* o) {
  for (int i = 0; i < 5; ++i) o[i] = s[1 + i];
  for (int i = 0; i < 6; ++i) o[5 + i] = clampd(s[6 + i], -10.0, 10.0);
}

}  // namespace mrl

#include "humanoid.h"
