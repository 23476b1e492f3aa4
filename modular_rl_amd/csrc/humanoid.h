// Humanoid-v2 (gym humanoid.xml) as 3-D articulated rigid-body dynamics, fp64 with FMA
// contraction off: the operation-for-operation twin of oracle/humanoid.py (see it for
// the model and the deviations from MuJoCo: compliant ground contact at the geoms' end
// caps and penalty joint limits instead of the constraint solver, semi-implicit Euler
// instead of RK4).  Com-based formulation (Featherstone in coordinates centred at the
// humanoid's COM, as MuJoCo's smooth dynamics): kinematics -> cinert / cdof / cvel /
// cdof_dot -> contact forces -> RNEA bias forces -> CRBA mass matrix -> tree-sparse
// L^T D L solve -> integrate.
//
// ONE WAVE PER ENV, its state in LDS (Wave): every phase spreads over the lanes what
// is independent -- bodies' local poses and inertias, dofs' axes and mass-matrix
// rows, the 29 contact spheres, the L^T D L updates of one pivot, the solves' column
// updates -- and walks tree levels or pivots in sequence where the algorithm is
// sequential.  Each element is computed by the same expression, in the same order, as
// in the numpy twin.  A wave's LDS operations complete in issue order, so the phases
// need compiler fences only (WAVE_SYNC), no barriers.
// Model constants: humanoid_model.h (generated from modular_rl_amd/humanoid_model.py).
#pragma once
#include "humanoid_model.h"
#include "mrl_common.h"

#pragma clang fp contract(off)

namespace mrl {
namespace hm {

constexpr double DT = 0.003, GRAV = 9.81;
constexpr int FRAME_SKIP = 5;
constexpr double KC = 20000.0, CC = 400.0, CF = 1000.0, MU = 1.0, KL = 2000.0, CL = 5.0;
constexpr double CTRL_LIMIT = 0.4, INIT_Z = 1.4;
constexpr int NS = NQ + NV + NACT, OBS = 376, NU = 48;

__device__ inline void cross3(const double* a, const double* b, double* r) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
// R row-major [9]
__device__ inline void mv3(const double* R, const double* v, double* r) {
#pragma unroll
  for (int i = 0; i < 3; ++i) r[i] = (R[3 * i] * v[0] + R[3 * i + 1] * v[1]) + R[3 * i + 2] * v[2];
}
__device__ inline void mm3(const double* A, const double* B, double* r) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) r[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}
__device__ inline void quat_mat(double w, double x, double y, double z, double* R) {
  R[0] = 1.0 - 2.0 * (y * y + z * z);
  R[1] = 2.0 * (x * y - w * z);
  R[2] = 2.0 * (x * z + w * y);
  R[3] = 2.0 * (x * y + w * z);
  R[4] = 1.0 - 2.0 * (x * x + z * z);
  R[5] = 2.0 * (y * z - w * x);
  R[6] = 2.0 * (x * z - w * y);
  R[7] = 2.0 * (y * z + w * x);
  R[8] = 1.0 - 2.0 * (x * x + y * y);
}
__device__ inline void axis_rot(const double* a, double s, double c, double* R) {
  const double t = 1.0 - c;
  R[0] = t * a[0] * a[0] + c;
  R[1] = t * a[0] * a[1] - s * a[2];
  R[2] = t * a[0] * a[2] + s * a[1];
  R[3] = t * a[0] * a[1] + s * a[2];
  R[4] = t * a[1] * a[1] + c;
  R[5] = t * a[1] * a[2] - s * a[0];
  R[6] = t * a[0] * a[2] - s * a[1];
  R[7] = t * a[1] * a[2] + s * a[0];
  R[8] = t * a[2] * a[2] + c;
}
__device__ inline void cross_motion(const double* v, const double* u, double* r) {
  double l1[3], l2[3];
  cross3(v, u, r);
  cross3(v, u + 3, l1);
  cross3(v + 3, u, l2);
#pragma unroll
  for (int i = 0; i < 3; ++i) r[3 + i] = l1[i] + l2[i];
}
__device__ inline void cross_force(const double* v, const double* f, double* r) {
  double t1[3], t2[3];
  cross3(v, f, t1);
  cross3(v + 3, f + 3, t2);
#pragma unroll
  for (int i = 0; i < 3; ++i) r[i] = t1[i] + t2[i];
  cross3(v, f + 3, r + 3);
}
__device__ inline void mul_inert(const double* I, const double* v, double* r) {
  double mdl[3], wmd[3];
  cross3(I + 6, v + 3, mdl);
  r[0] = ((I[0] * v[0] + I[3] * v[1]) + I[4] * v[2]) + mdl[0];
  r[1] = ((I[3] * v[0] + I[1] * v[1]) + I[5] * v[2]) + mdl[1];
  r[2] = ((I[4] * v[0] + I[5] * v[1]) + I[2] * v[2]) + mdl[2];
  cross3(v, I + 6, wmd);
#pragma unroll
  for (int i = 0; i < 3; ++i) r[3 + i] = I[9] * v[3 + i] + wmd[i];
}
__device__ inline double dot6(const double* a, const double* b) {
  return ((((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3]) + a[4] * b[4]) + a[5] * b[5];
}

#define WAVE_SYNC() asm volatile("" ::: "memory")

// one env's working state (LDS, one wave)
struct Wave {
  double s[NQ + NV + NACT];  // qpos ++ qvel ++ ctrl
  double Qloc[NB][9], oloc[NB][3], lax[17][3], lanc[17][3];
  double R[NB][9], xpos[NB][3], xipos[NB][3], haxis[17][3], hanchor[17][3], com[3];
  double cinert[NB][10], cdof[NV][6], cdof_dot[NV][6], cvel[NB][6];
  double fsph[NSPH][6], cfrc[NB][6], cacc[NB][6], fb[NB][6], crb[NB][10];
  double L[NV][NV], x[NV];
  double red[2];
};

// kinematics, com-based inertias / axes / velocities and contact forces of W.s
__device__ inline void forward(Wave& W, int lane) {
  const double* q = W.s;
  const double* qd = W.s + NQ;
  // each body's pose in its parent's frame (after its hinges), all bodies at once
  if (lane >= 1 && lane < NB) {
    const int b = lane;
    double Q[9], o[3];
    quat_mat(BODY_QUAT[4 * b], BODY_QUAT[4 * b + 1], BODY_QUAT[4 * b + 2], BODY_QUAT[4 * b + 3], Q);
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = BODY_POS[3 * b + i];
    for (int j = BODY_HINGE0[b]; j < BODY_HINGE0[b] + BODY_NHINGE[b]; ++j) {
      const double* ax = &HINGE_AXIS[3 * j];
      const double* jp = &HINGE_POS[3 * j];
      double ra[3], rot[9], Qn[9], rb[3];
      mv3(Q, jp, ra);
#pragma unroll
      for (int i = 0; i < 3; ++i) W.lanc[j][i] = o[i] + ra[i];
      mv3(Q, ax, W.lax[j]);
      double sn, cs;
      sincos(q[7 + j], &sn, &cs);
      axis_rot(ax, sn, cs, rot);
      mm3(Q, rot, Qn);
#pragma unroll
      for (int i = 0; i < 9; ++i) Q[i] = Qn[i];
      mv3(Q, jp, rb);
#pragma unroll
      for (int i = 0; i < 3; ++i) o[i] = W.lanc[j][i] - rb[i];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) W.Qloc[b][i] = Q[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) W.oloc[b][i] = o[i];
  } else if (lane == 0) {
    const double qn = sqrt(((q[3] * q[3] + q[4] * q[4]) + q[5] * q[5]) + q[6] * q[6]);
    quat_mat(q[3] / qn, q[4] / qn, q[5] / qn, q[6] / qn, W.R[0]);
    W.xpos[0][0] = q[0];
    W.xpos[0][1] = q[1];
    W.xpos[0][2] = q[2];
  }
  WAVE_SYNC();
  // world poses, root -> leaves (one tree level at a time)
  for (int lv = 1; lv < NLEVEL; ++lv) {
    const int n = LEVEL_START[lv + 1] - LEVEL_START[lv];
    if (lane < n) {
      const int b = LEVEL_BODIES[LEVEL_START[lv] + lane];
      const int p = BODY_PARENT[b];
      double off[3];
      mm3(W.R[p], W.Qloc[b], W.R[b]);
      mv3(W.R[p], W.oloc[b], off);
#pragma unroll
      for (int i = 0; i < 3; ++i) W.xpos[b][i] = W.xpos[p][i] + off[i];
      for (int j = BODY_HINGE0[b]; j < BODY_HINGE0[b] + BODY_NHINGE[b]; ++j) {
        double ra[3];
        mv3(W.R[p], W.lax[j], W.haxis[j]);
        mv3(W.R[p], W.lanc[j], ra);
#pragma unroll
        for (int i = 0; i < 3; ++i) W.hanchor[j][i] = W.xpos[p][i] + ra[i];
      }
    }
    WAVE_SYNC();
  }
  if (lane < NB) {
    double ri[3];
    mv3(W.R[lane], &BODY_IPOS[3 * lane], ri);
#pragma unroll
    for (int i = 0; i < 3; ++i) W.xipos[lane][i] = W.xpos[lane][i] + ri[i];
  }
  WAVE_SYNC();
  if (lane < 3) {
    double acc = 0.0;
    for (int b = 0; b < NB; ++b) acc = acc + BODY_MASS[b] * W.xipos[b][lane];
    W.com[lane] = acc / TOTAL_MASS;
  }
  WAVE_SYNC();
  if (lane < NB) {  // cinert
    const int b = lane;
    const double* I6 = &BODY_INERTIA[6 * b];
    const double Ib[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
    double Rt[9], T[9], Iw[9], d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Rt[3 * i + j] = W.R[b][3 * j + i];
    mm3(W.R[b], Ib, T);
    mm3(T, Rt, Iw);
    const double m = BODY_MASS[b];
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = W.xipos[b][i] - W.com[i];
    double* ci = W.cinert[b];
    ci[0] = Iw[0] + m * (d[1] * d[1] + d[2] * d[2]);
    ci[1] = Iw[4] + m * (d[0] * d[0] + d[2] * d[2]);
    ci[2] = Iw[8] + m * (d[0] * d[0] + d[1] * d[1]);
    ci[3] = Iw[1] - m * (d[0] * d[1]);
    ci[4] = Iw[2] - m * (d[0] * d[2]);
    ci[5] = Iw[5] - m * (d[1] * d[2]);
    ci[6] = m * d[0];
    ci[7] = m * d[1];
    ci[8] = m * d[2];
    ci[9] = m;
  } else if (lane >= 32 && lane < 32 + NV) {  // cdof
    const int i = lane - 32;
    double* cd = W.cdof[i];
    if (i < 3) {
#pragma unroll
      for (int k = 0; k < 6; ++k) cd[k] = (k == 3 + i) ? 1.0 : 0.0;
    } else {
      double off[3];
      if (i < 6) {
        cd[0] = W.R[0][i - 3];
        cd[1] = W.R[0][3 + i - 3];
        cd[2] = W.R[0][6 + i - 3];
#pragma unroll
        for (int k = 0; k < 3; ++k) off[k] = W.com[k] - W.xpos[0][k];
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          cd[k] = W.haxis[i - 6][k];
          off[k] = W.com[k] - W.hanchor[i - 6][k];
        }
      }
      cross3(cd, off, cd + 3);
    }
  }
  WAVE_SYNC();
  // cvel and cdof_dot (MuJoCo mj_comVel order), root -> leaves
  if (lane == 0) {
    double cv[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      W.cdof_dot[0][i] = W.cdof_dot[1][i] = W.cdof_dot[2][i] = 0.0;
      cv[i] = 0.0 + ((W.cdof[0][i] * qd[0] + W.cdof[1][i] * qd[1]) + W.cdof[2][i] * qd[2]);
    }
#pragma unroll
    for (int k = 3; k < 6; ++k) cross_motion(cv, W.cdof[k], W.cdof_dot[k]);
#pragma unroll
    for (int i = 0; i < 6; ++i)
      W.cvel[0][i] = cv[i] + ((W.cdof[3][i] * qd[3] + W.cdof[4][i] * qd[4]) + W.cdof[5][i] * qd[5]);
  }
  WAVE_SYNC();
  for (int lv = 1; lv < NLEVEL; ++lv) {
    const int n = LEVEL_START[lv + 1] - LEVEL_START[lv];
    if (lane < n) {
      const int b = LEVEL_BODIES[LEVEL_START[lv] + lane];
      double cv[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) cv[i] = W.cvel[BODY_PARENT[b]][i];
      for (int d = 6 + BODY_HINGE0[b]; d < 6 + BODY_HINGE0[b] + BODY_NHINGE[b]; ++d) {
        cross_motion(cv, W.cdof[d], W.cdof_dot[d]);
#pragma unroll
        for (int i = 0; i < 6; ++i) cv[i] = cv[i] + W.cdof[d][i] * qd[d];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) W.cvel[b][i] = cv[i];
    }
    WAVE_SYNC();
  }
  // ground contact: sphere s of body b against z = 0, at the sphere's lowest point
  if (lane < NSPH) {
    const int s = lane;
    const int b = SPHERE_BODY[s];
    const double r = SPHERE_R[s];
    double cs[3], c[3], rel[3], wr[3], v[3], fv[3];
    mv3(W.R[b], &SPHERE_POS[3 * s], cs);
#pragma unroll
    for (int i = 0; i < 3; ++i) c[i] = W.xpos[b][i] + cs[i];
    const double pen = r - c[2];
    rel[0] = c[0] - W.com[0];
    rel[1] = c[1] - W.com[1];
    rel[2] = (c[2] - r) - W.com[2];
    cross3(W.cvel[b], rel, wr);
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = W.cvel[b][3 + i] + wr[i];
    const double fnr = KC * pen - CC * v[2];
    const double fn = pen > 0.0 ? (fnr > 0.0 ? fnr : 0.0) : 0.0;
    const double fx = -(CF * v[0]);
    const double fy = -(CF * v[1]);
    const double mag = sqrt(fx * fx + fy * fy);
    const double lim = MU * fn;
    const double sc = mag > lim ? lim / (mag > 0.0 ? mag : 1.0) : 1.0;
    fv[0] = fx * sc;
    fv[1] = fy * sc;
    fv[2] = fn;
    cross3(rel, fv, W.fsph[s]);
#pragma unroll
    for (int i = 0; i < 3; ++i) W.fsph[s][3 + i] = fv[i];
  }
  WAVE_SYNC();
  if (lane < NB) {  // per body, its spheres in order
    const int b = lane;
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int s = BODY_SPH0[b]; s < BODY_SPH0[b] + BODY_NSPH[b]; ++s)
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[i] = acc[i] + W.fsph[s][i];
#pragma unroll
    for (int i = 0; i < 6; ++i) W.cfrc[b][i] = acc[i];
  }
  WAVE_SYNC();
}

__device__ inline double clamp_ctrl(double c) { return c < -CTRL_LIMIT ? -CTRL_LIMIT : (c > CTRL_LIMIT ? CTRL_LIMIT : c); }

// gear * clip(ctrl) at dof i (0 for the unactuated root dofs)
__device__ inline double actuator_force(const double* ctrl, int i) {
  double f = 0.0;
  for (int k = 0; k < NACT; ++k)
    if (ACT_DOF[k] == i) f = ACT_GEAR[k] * clamp_ctrl(ctrl[k]);
  return f;
}

// W.x <- qdd of M qdd = qfrc_actuator + passive + limits - (bias - contact); needs forward(W)
__device__ inline void accelerations(Wave& W, int lane) {
  const double* q = W.s;
  const double* qd = W.s + NQ;
  const double* ctrl = W.s + NQ + NV;
  if (lane == 0) {
    double ca[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0 + GRAV};
#pragma unroll
    for (int k = 3; k < 6; ++k)
#pragma unroll
      for (int i = 0; i < 6; ++i) ca[i] = ca[i] + W.cdof_dot[k][i] * qd[k];
#pragma unroll
    for (int i = 0; i < 6; ++i) W.cacc[0][i] = ca[i];
  }
  WAVE_SYNC();
  for (int lv = 1; lv < NLEVEL; ++lv) {
    const int n = LEVEL_START[lv + 1] - LEVEL_START[lv];
    if (lane < n) {
      const int b = LEVEL_BODIES[LEVEL_START[lv] + lane];
      double ca[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) ca[i] = W.cacc[BODY_PARENT[b]][i];
      for (int d = 6 + BODY_HINGE0[b]; d < 6 + BODY_HINGE0[b] + BODY_NHINGE[b]; ++d)
#pragma unroll
        for (int i = 0; i < 6; ++i) ca[i] = ca[i] + W.cdof_dot[d][i] * qd[d];
#pragma unroll
      for (int i = 0; i < 6; ++i) W.cacc[b][i] = ca[i];
    }
    WAVE_SYNC();
  }
  if (lane < NB) {
    const int b = lane;
    double Ia[6], Iv[6], cf[6];
    mul_inert(W.cinert[b], W.cacc[b], Ia);
    mul_inert(W.cinert[b], W.cvel[b], Iv);
    cross_force(W.cvel[b], Iv, cf);
#pragma unroll
    for (int i = 0; i < 6; ++i) W.fb[b][i] = (Ia[i] + cf[i]) - W.cfrc[b][i];
#pragma unroll
    for (int i = 0; i < 10; ++i) W.crb[b][i] = W.cinert[b][i];
  }
  WAVE_SYNC();
  // subtree sums, leaves -> root: a parent adds its children in descending index
  for (int lv = NLEVEL - 2; lv >= 0; --lv) {
    const int n = LEVEL_START[lv + 1] - LEVEL_START[lv];
    if (lane < n) {
      const int p = LEVEL_BODIES[LEVEL_START[lv] + lane];
      for (int c = CHILD_START[p]; c < CHILD_START[p + 1]; ++c) {
        const int ch = CHILDREN[c];
#pragma unroll
        for (int i = 0; i < 6; ++i) W.fb[p][i] = W.fb[p][i] + W.fb[ch][i];
#pragma unroll
        for (int i = 0; i < 10; ++i) W.crb[p][i] = W.crb[p][i] + W.crb[ch][i];
      }
    }
    WAVE_SYNC();
  }
  // mass-matrix row i over its ancestors, and the generalised force
  if (lane < NV) {
    const int i = lane;
    double F[6];
    mul_inert(W.crb[DOF_BODY[i]], W.cdof[i], F);
    for (int j = i; j >= 0; j = DOF_PARENT[j]) W.L[i][j] = dot6(W.cdof[j], F);
    if (i >= 6) W.L[i][i] = W.L[i][i] + HINGE_ARM[i - 6];
    const double bias = dot6(W.cdof[i], W.fb[DOF_BODY[i]]);
    double t = actuator_force(ctrl, i) - bias;
    if (i >= 6) {
      const int j = i - 6;
      const double qj = q[7 + j], vj = qd[i];
      const double lo = HINGE_LO[j], hi = HINGE_HI[j];
      const double lim = qj < lo ? KL * (lo - qj) - CL * vj : (qj > hi ? KL * (hi - qj) - CL * vj : 0.0);
      const double passive = (-(HINGE_STIFF[j] * qj) - HINGE_DAMP[j] * vj) + lim;
      t = t + passive;
    }
    W.x[i] = t;
  }
  WAVE_SYNC();
  // L^T D L, leaves first: pivot k updates every (ancestor i, ancestor-or-self j of i)
  // pair from its still unscaled row, then scales its row
  for (int k = NV - 1; k >= 0; --k) {
    const double invd = 1.0 / W.L[k][k];
    for (int pp = LDL_START[k] + lane; pp < LDL_START[k + 1]; pp += 64) {
      const int i = LDL_I[pp], j = LDL_J[pp];
      W.L[i][j] = W.L[i][j] - W.L[k][i] * (W.L[k][j] * invd);
    }
    WAVE_SYNC();
    int i = DOF_PARENT[k];
    for (int a = 0; a < lane && i >= 0; ++a) i = DOF_PARENT[i];  // the lane-th ancestor
    if (i >= 0) W.L[k][i] = W.L[k][i] * invd;
    WAVE_SYNC();
  }
  // L^T y = x (leaves first), D z = y, L x = z (column by column)
  for (int i = NV - 1; i >= 0; --i) {
    int j = DOF_PARENT[i];
    for (int a = 0; a < lane && j >= 0; ++a) j = DOF_PARENT[j];
    if (j >= 0) W.x[j] = W.x[j] - W.L[i][j] * W.x[i];
    WAVE_SYNC();
  }
  if (lane < NV) W.x[lane] = W.x[lane] / W.L[lane][lane];
  WAVE_SYNC();
  for (int j = 0; j < NV; ++j) {
    const int pp = DESC_START[j] + lane;
    if (pp < DESC_START[j + 1]) {
      const int i = DESC[pp];
      W.x[i] = W.x[i] - W.L[i][j] * W.x[j];
    }
    WAVE_SYNC();
  }
}

// one dt in place on W.s; returns the COM x of the state it started from
__device__ inline double substep(Wave& W, int lane) {
  forward(W, lane);
  const double com_x = W.com[0];
  accelerations(W, lane);
  double* q = W.s;
  double* qd = W.s + NQ;
  if (lane < NV) qd[lane] = qd[lane] + DT * W.x[lane];
  WAVE_SYNC();
  if (lane < 3) {
    q[lane] = q[lane] + DT * qd[lane];
  } else if (lane == 3) {
    const double w0 = qd[3], w1 = qd[4], w2 = qd[5];
    const double nw = sqrt((w0 * w0 + w1 * w1) + w2 * w2);
    const double half = (0.5 * DT) * nw;
    const double sh = nw > 0.0 ? sin(half) / (nw > 0.0 ? nw : 1.0) : 0.0;
    const double ch = cos(half);
    const double dq[4] = {ch, w0 * sh, w1 * sh, w2 * sh};
    const double a0 = q[3], a1 = q[4], a2 = q[5], a3 = q[6];
    const double qw = ((a0 * dq[0] - a1 * dq[1]) - a2 * dq[2]) - a3 * dq[3];
    const double qx = ((a0 * dq[1] + a1 * dq[0]) + a2 * dq[3]) - a3 * dq[2];
    const double qy = ((a0 * dq[2] - a1 * dq[3]) + a2 * dq[0]) + a3 * dq[1];
    const double qz = ((a0 * dq[3] + a1 * dq[2]) - a2 * dq[1]) + a3 * dq[0];
    const double n = sqrt(((qw * qw + qx * qx) + qy * qy) + qz * qz);
    q[3] = qw / n;
    q[4] = qx / n;
    q[5] = qy / n;
    q[6] = qz / n;
  } else if (lane >= 8 && lane < 8 + 17) {
    const int j = lane - 8;
    q[7 + j] = q[7 + j] + DT * qd[6 + j];
  }
  WAVE_SYNC();
  return com_x;
}

// reward and done of a step that started at COM x x_before; needs forward(W) of the
// new state.  reward = 0.25 dx_com / dt + 5 - 0.1 |ctrl|^2 - min(0.5e-6 |cfrc_ext|^2, 10)
__device__ inline void reward_done(Wave& W, int lane, double x_before, double& rew, bool& done) {
  const double* ctrl = W.s + NQ + NV;
  if (lane == 0) {
    double asq = 0.0;
    for (int j = 0; j < NACT; ++j) asq = asq + ctrl[j] * ctrl[j];
    double csq = 0.0;
    for (int b = 0; b < NB; ++b)
      for (int k = 0; k < 6; ++k) csq = csq + W.cfrc[b][k] * W.cfrc[b][k];
    const double ic = 0.5e-6 * csq;
    const double impact = ic < 10.0 ? ic : 10.0;
    W.red[0] = ((0.25 * (W.com[0] - x_before) / DT - 0.1 * asq) - impact) + 5.0;
  }
  const bool fin = lane < NS ? isfinite(W.s[lane]) : true;
  const bool all_fin = __ballot(!fin) == 0;
  WAVE_SYNC();
  rew = W.red[0];
  done = !(all_fin && (W.s[2] >= 1.0) && (W.s[2] <= 2.0));
}

// reset (core.py:186 / gym reset_model): qpos0 + U(-.01, .01) (quaternion included),
// qvel U(-.01, .01), ctrl 0, from the Philox uniforms of (gid, episode w) on domain 1
__device__ inline void reset(Wave& W, int lane, uint64_t seed, uint32_t gid, uint64_t w) {
  double* u = W.L[0];  // scratch for the 48 uniforms
  if (lane < NU / 2) philox_uniform2(seed, 1, gid, w, (uint32_t)lane, u[2 * lane], u[2 * lane + 1]);
  WAVE_SYNC();
  if (lane < NQ) {
    double v = u[lane] * 0.02 - 0.01;
    if (lane == 2) v = v + INIT_Z;
    if (lane == 3) v = v + 1.0;
    W.s[lane] = v;
  } else if (lane < NQ + NV) {
    W.s[lane] = u[lane] * 0.02 - 0.01;
  } else if (lane < NS) {
    W.s[lane] = 0.0;
  }
  WAVE_SYNC();
}

// the 376-d observation through out(k, value), lanes splitting the entries; needs
// forward(W): qpos[2:] | qvel | cinert | cvel | qfrc_actuator | cfrc_ext (world: 0)
template <class Out>
__device__ inline void observation(const Wave& W, int lane, Out out) {
  for (int k = lane; k < OBS; k += 64) {
    double v;
    if (k < 22) {
      v = W.s[2 + k];
    } else if (k < 45) {
      v = W.s[NQ + k - 22];
    } else if (k < 185) {
      const int b = (k - 45) / 10 - 1, c = (k - 45) % 10;
      v = b < 0 ? 0.0 : W.cinert[b][c];
    } else if (k < 269) {
      const int b = (k - 185) / 6 - 1, c = (k - 185) % 6;
      v = b < 0 ? 0.0 : W.cvel[b][c];
    } else if (k < 292) {
      v = actuator_force(W.s + NQ + NV, k - 269);
    } else {
      const int b = (k - 292) / 6 - 1, c = (k - 292) % 6;
      v = b < 0 ? 0.0 : W.cfrc[b][c];
    }
    out(k, v);
  }
}

}  // namespace hm

constexpr int HM_NQ = hm::NQ, HM_NV = hm::NV, HM_ACT = hm::NACT, HM_NS = hm::NS, HM_OBS = hm::OBS, HM_NU = hm::NU;

}  // namespace mrl
