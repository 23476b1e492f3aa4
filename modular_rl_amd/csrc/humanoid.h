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
#include <cstddef>

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
constexpr int NHINGE = NV - 6;  // the hinge dofs follow the free joint's 6

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
#define HM_INLINE __device__ __attribute__((always_inline)) inline
// diagnostic phase stamps (shader clock) into st[k] when st is set -- never in production
#define HM_STAMP(k)                                                                     \
  do {                                                                                  \
    if (st != nullptr && lane == 0) st[k] = (int64_t)__builtin_amdgcn_s_memtime();      \
  } while (0)

// The model's index tables and constants, built at compile time (SHARED) and copied
// into each block's LDS (Shared) at launch: a phase reads its table word or constant
// with a ds_read issued ahead of its data instead of a lane-indexed global load (a
// round trip of ~1k cycles each), and the sequential walks stay rolled loops -- the
// step's loop body must fit the instruction cache (fully unrolled it did not: 4.5 ms
// per step instead of 0.9).  Index tables are packed bytes, NONE = no entry.
constexpr uint32_t NONE = 0xff;
HM_INLINE uint32_t byte_of(uint32_t w, int s) { return (w >> (8 * s)) & 0xffu; }

constexpr int N_ENT = NV + 170;               // mass-matrix entries (i, j in {i} + ancestors(i)); bound checked below
constexpr int W_SUB = 0;                      // [NLEVEL] level lv's body at this lane | its children << 8, 16, 24
constexpr int W_PATH = W_SUB + NLEVEL;        // [2] body `lane`'s path below the root, root side first (bytes)
constexpr int W_OWN = W_PATH + 2;             // body `lane`: hinge0 | nhinge << 8 | sph0 << 16 | nsph << 24
constexpr int W_MISC = W_OWN + 1;             // dof `lane`'s body | sphere `lane`'s body << 8 | hinge `lane - 32`'s parent body << 16
constexpr int W_ENT = W_MISC + 1;             // [ceil(N_ENT/128)] mass-matrix entries r, r+64: i | j << 8 (, << 16, 24)
constexpr int N_ENT_WORDS = (N_ENT + 127) / 128;
constexpr int PATH_LEN = NLEVEL - 1;
// The hinge dofs along body b's path below the root (root side first, each body's hinges
// in order) as bytes: dof | own << 5 | own hinge index << 6, padding 0xff (dof field 31)
constexpr int path_dof_count(int b) {
  int n = 0;
  for (int a = b; a > 0; a = BODY_PARENT[a]) n += BODY_NHINGE[a];
  return n;
}
constexpr int max_path_dofs() {
  int n = 0;
  for (int b = 0; b < NB; ++b) n = path_dof_count(b) > n ? path_dof_count(b) : n;
  return n;
}
constexpr int MAXPD = max_path_dofs();
constexpr int PD_WORDS = (MAXPD + 3) / 4;

// Branch-parallel L^T D L schedule.  The dof tree is a trunk (a chain 0 .. NT-1 of dofs
// with two or more leaves below) carrying branches (chains NT .. NV-1 hanging off trunk
// dofs: the legs and the arms).  A branch pivot k updates pairs (i, j) of its ancestors:
// entries with i in k's branch belong to that branch alone, entries with i in the trunk
// are shared by every branch below i.  So the branches' pivots run in lockstep (step s:
// each branch's s-th pivot from its leaf, 16 lanes per branch), updating their branch
// entries in place and leaving their trunk-entry products p_k(i, j) in C; one gather then
// subtracts them from each trunk entry in descending k, and the trunk pivots follow in
// sequence -- every entry sees the same operations in the same order as the pivot-by-pivot
// loop.  Item words (dst | a1 << 11 | a2 << 21 | sub << 31, offsets in doubles from
// W.L): dst = dst - a1 (a2 invd) if sub, else dst = a1 (a2 invd); a row scaling is
// a1 = L[k][a] times a2 = the ONE slot (1 invd = invd exactly).
constexpr int dof_leaves(int d) {
  int n = 0;
  for (int c = d + 1; c < NV; ++c)
    if (DOF_PARENT[c] == d) n += dof_leaves(c);
  return n > 0 ? n : 1;
}
constexpr int trunk_len() {
  int n = 0;
  while (n < NV && dof_leaves(n) >= 2) ++n;
  return n;
}
constexpr int NT = trunk_len();                  // trunk dofs 0 .. NT-1
constexpr int NTP = NT * (NT + 1) / 2;           // trunk entries (i, j <= i)
constexpr int NCONTRIB = (NV - NT) * NTP;        // C: [branch pivot k - NT][trunk entry]
constexpr int OFF_ONE = NV * NV, OFF_C = OFF_ONE + 1, OFF_JUNK = OFF_C + NCONTRIB;
constexpr int branch_count() {
  int n = 0;
  for (int d = NT; d < NV; ++d) n += DOF_PARENT[d] < NT ? 1 : 0;
  return n;
}
constexpr int NBRANCH = branch_count();
constexpr int branch_root(int b) {
  for (int d = NT; d < NV; ++d)
    if (DOF_PARENT[d] < NT && b-- == 0) return d;
  return -1;
}
constexpr int branch_leaf(int b) { return b + 1 < NBRANCH ? branch_root(b + 1) - 1 : NV - 1; }
constexpr int anc_count(int k) {
  int n = 0;
  for (int l = 0; l < 16; ++l) n += ANC[16 * k + l] >= 0 ? 1 : 0;
  return n;
}
constexpr int ldl_items(int k) { return (LDL_START[k + 1] - LDL_START[k]) + anc_count(k); }
constexpr int branch_steps() {
  int n = 0;
  for (int b = 0; b < NBRANCH; ++b) n = branch_leaf(b) - branch_root(b) + 1 > n ? branch_leaf(b) - branch_root(b) + 1 : n;
  return n;
}
constexpr int NBSTEP = branch_steps();
constexpr int branch_slots() {
  int n = 0;
  for (int k = NT; k < NV; ++k) n = (ldl_items(k) + 15) / 16 > n ? (ldl_items(k) + 15) / 16 : n;
  return n;
}
constexpr int NBSLOT = branch_slots();         // item words per lane and step (+1: the pivot's diagonal)
constexpr int W_BR = W_ENT + N_ENT_WORDS;      // [NBSTEP][NBSLOT + 1] branch-step item words, then k NV + k
constexpr int W_TG = W_BR + NBSTEP * (NBSLOT + 1);  // trunk entry `lane`: i NV + j | branch pivots below i << 16
constexpr int W_PDOF = W_TG + 1;                    // [PD_WORDS] body (lane & 15)'s path dofs (bytes)
constexpr int W_TR = W_PDOF + PD_WORDS;             // [NT] trunk pivot k's item at this lane (one per lane)
// the lane of trunk pivot k's item on the next pivot's diagonal (k - 1, k - 1), packed 6
// bits per pivot (k >= 1; the trunk is a chain, so k - 1 is k's parent)
constexpr uint64_t trunk_diag_lanes() {
  uint64_t m = 0;
  for (int k = 1; k < NT; ++k)
    for (int pp = LDL_START[k]; pp < LDL_START[k + 1]; ++pp)
      if (LDL_I[pp] == k - 1 && LDL_J[pp] == k - 1) m |= (uint64_t)(pp - LDL_START[k]) << (6 * k);
  return m;
}
constexpr uint64_t TRUNK_DIAG_LANES = trunk_diag_lanes();
constexpr int TOPO_WORDS = W_TR + NT;
constexpr bool ldl_schedule_fits() {
  for (int d = 0; d < NT; ++d)
    if (d > 0 && DOF_PARENT[d] != d - 1) return false;  // the trunk is a chain
  for (int d = NT; d < NV; ++d) {
    if (dof_leaves(d) != 1) return false;
    if (DOF_PARENT[d] >= NT && DOF_PARENT[d] != d - 1) return false;  // branches are chains
  }
  for (int k = 0; k < NT; ++k)
    if (ldl_items(k) > 64) return false;  // a trunk pivot's items take one lane each
  return NT >= 1 && NBRANCH >= 1 && NBRANCH <= 4 && NV - NT <= 16 && NTP <= 64 && OFF_JUNK + 64 <= 2048 &&
         OFF_ONE < 1024;
}

struct Shared {
  uint32_t w[TOPO_WORDS][64];
  double quat[NB][4], pos[NB][3], ipos[NB][3], inertia[NB][6], mass[NB];
  double hax[NHINGE][3], hpos[NHINGE][3], lo[NHINGE], hi[NHINGE], stiff[NHINGE], damp[NHINGE], arm[NHINGE];
  double sph_pos[NSPH][3], sph_r[NSPH], gear[NACT];
  uint8_t hinge0[NB], nhinge[NB], act_of_dof[NV];  // act_of_dof: NONE for the root dofs
};

// strict-ancestor / strict-descendant bit masks of each dof
constexpr uint32_t anc_mask(int i) {
  uint32_t m = 0;
  for (int j = DOF_PARENT[i]; j >= 0; j = DOF_PARENT[j]) m |= 1u << j;
  return m;
}
constexpr uint32_t desc_mask(int j) {
  uint32_t m = 0;
  for (int i = 0; i < NV; ++i)
    if ((anc_mask(i) >> j) & 1u) m |= 1u << i;
  return m;
}
constexpr int n_entries() {
  int n = 0;
  for (int i = 0; i < NV; ++i) {
    ++n;
    for (int j = DOF_PARENT[i]; j >= 0; j = DOF_PARENT[j]) ++n;
  }
  return n;
}
constexpr int body_depth(int b) {
  int d = 0;
  for (int a = BODY_PARENT[b]; a >= 0; a = BODY_PARENT[a]) ++d;
  return d;
}
constexpr bool topo_fits() {
  for (int b = 0; b < NB; ++b) {
    if (CHILD_START[b + 1] - CHILD_START[b] > 3 || BODY_NHINGE[b] > 3 || body_depth(b) > PATH_LEN || body_depth(b) > 8) return false;
    if (BODY_PARENT[b] >= b) return false;  // parents first
  }
  for (int k = 0; k < NV; ++k)
    if (LDL_START[k + 1] - LDL_START[k] > 128) return false;
  for (int lv = 0; lv < NLEVEL; ++lv)  // the subtree sums take four parents of a level per wave
    if (LEVEL_START[lv + 1] - LEVEL_START[lv] > 4) return false;
  return NV <= 32 && NB <= 32 && NSPH <= 64 && NACT <= 64 && NHINGE <= 32 && n_entries() <= N_ENT;
}
static_assert(topo_fits(), "humanoid tree exceeds the wave layout");
static_assert(ldl_schedule_fits(), "humanoid dof tree does not fit the branch-parallel L^T D L schedule");
constexpr uint32_t ldl_item(int dst, int a1, int a2, int sub) {
  return (uint32_t)dst | (uint32_t)a1 << 11 | (uint32_t)a2 << 21 | (uint32_t)sub << 31;
}
constexpr bool dof_is_anc(int i, int k) {  // i a strict ancestor of k
  for (int a = DOF_PARENT[k]; a >= 0; a = DOF_PARENT[a])
    if (a == i) return true;
  return false;
}

struct MaskTable {
  uint32_t anc[NV], desc[NV];
};
constexpr MaskTable make_masks() {
  MaskTable m{};
  for (int i = 0; i < NV; ++i) {
    m.anc[i] = anc_mask(i);
    m.desc[i] = desc_mask(i);
  }
  return m;
}
__device__ constexpr MaskTable MASKS = make_masks();

constexpr uint32_t bytes4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return a | b << 8 | c << 16 | d << 24; }
constexpr uint32_t nb(int v) { return v < 0 ? NONE : (uint32_t)v; }
constexpr int hinge_body(int j) {
  for (int b = 0; b < NB; ++b)
    if (j >= BODY_HINGE0[b] && j < BODY_HINGE0[b] + BODY_NHINGE[b]) return b;
  return -1;
}
constexpr Shared make_shared() {
  Shared t{};
  for (int lane = 0; lane < 64; ++lane) {
    for (int lv = 0; lv < NLEVEL; ++lv) {
      const int n = LEVEL_START[lv + 1] - LEVEL_START[lv];
      uint32_t u = bytes4(NONE, NONE, NONE, NONE);
      if (lane < n) {
        const int b = LEVEL_BODIES[LEVEL_START[lv] + lane];
        u = (uint32_t)b;
        for (int c = 0; c < 3; ++c)
          u |= (CHILD_START[b] + c < CHILD_START[b + 1] ? (uint32_t)CHILDREN[CHILD_START[b] + c] : NONE) << (8 * (c + 1));
      }
      t.w[W_SUB + lv][lane] = u;
    }
    uint32_t path[8] = {NONE, NONE, NONE, NONE, NONE, NONE, NONE, NONE};
    if (lane < NB) {
      const int d = body_depth(lane);
      int a = lane;
      for (int s = d - 1; s >= 0; --s, a = BODY_PARENT[a]) path[s] = (uint32_t)a;
    }
    t.w[W_PATH][lane] = bytes4(path[0], path[1], path[2], path[3]);
    t.w[W_PATH + 1][lane] = bytes4(path[4], path[5], path[6], path[7]);
    t.w[W_OWN][lane] = lane < NB ? bytes4((uint32_t)BODY_HINGE0[lane], (uint32_t)BODY_NHINGE[lane], (uint32_t)BODY_SPH0[lane],
                                          (uint32_t)BODY_NSPH[lane])
                                 : 0u;
    t.w[W_MISC][lane] = (lane < NV ? (uint32_t)DOF_BODY[lane] : 0u) | (lane < NSPH ? (uint32_t)SPHERE_BODY[lane] : 0u) << 8 |
                        (lane >= 32 && lane < 32 + NHINGE ? nb(BODY_PARENT[hinge_body(lane - 32)]) : 0u) << 16;
  }
  // mass-matrix entries, row by row (diagonal first, then the ancestors nearest first)
  uint32_t ent[N_ENT_WORDS * 128] = {};
  for (int r = 0; r < N_ENT_WORDS * 128; ++r) ent[r] = NONE | NONE << 8;
  int r = 0;
  for (int i = 0; i < NV; ++i) {
    ent[r++] = (uint32_t)i | (uint32_t)i << 8;
    for (int j = DOF_PARENT[i]; j >= 0; j = DOF_PARENT[j]) ent[r++] = (uint32_t)i | (uint32_t)j << 8;
  }
  for (int q = 0; q < N_ENT_WORDS; ++q)
    for (int lane = 0; lane < 64; ++lane) t.w[W_ENT + q][lane] = ent[128 * q + lane] | ent[128 * q + 64 + lane] << 16;
  for (int lane = 0; lane < 64; ++lane) {
    uint8_t pd[PD_WORDS * 4] = {};
    for (int t = 0; t < PD_WORDS * 4; ++t) pd[t] = 0xff;
    const int b = lane & 15;
    if (b < NB) {
      int chain[8] = {}, n = 0, t = 0;
      for (int a = b; a > 0; a = BODY_PARENT[a]) chain[n++] = a;
      for (int s = n - 1; s >= 0; --s)
        for (int c = 0; c < BODY_NHINGE[chain[s]]; ++c)
          pd[t++] = (uint8_t)((6 + BODY_HINGE0[chain[s]] + c) | (chain[s] == b ? 0x20 | c << 6 : 0));
    }
    for (int q = 0; q < PD_WORDS; ++q) t.w[W_PDOF + q][lane] = bytes4(pd[4 * q], pd[4 * q + 1], pd[4 * q + 2], pd[4 * q + 3]);
  }
  // branch-parallel L^T D L: step st, lane 16 b + l runs items l, l + 16, ... of branch b's
  // st-th pivot from its leaf (pairs in LDL order, then the row scalings); idle slots
  // write the lane's junk slot
  for (int st = 0; st < NBSTEP; ++st)
    for (int lane = 0; lane < 64; ++lane) {
      for (int q = 0; q < NBSLOT; ++q) t.w[W_BR + st * (NBSLOT + 1) + q][lane] = ldl_item(OFF_JUNK + lane, 0, 0, 0);
      t.w[W_BR + st * (NBSLOT + 1) + NBSLOT][lane] = 0u;
    }
  for (int b = 0; b < NBRANCH; ++b)
    for (int st = 0; st < NBSTEP; ++st) {
      const int k = branch_leaf(b) - st;
      if (k < branch_root(b)) continue;
      int q = 0;
      for (int pp = LDL_START[k]; pp < LDL_START[k + 1]; ++pp, ++q) {
        const int i = LDL_I[pp], j = LDL_J[pp];
        t.w[W_BR + st * (NBSLOT + 1) + q / 16][16 * b + q % 16] =
            i >= NT ? ldl_item(i * NV + j, k * NV + i, k * NV + j, 1)
                    : ldl_item(OFF_C + (k - NT) * NTP + i * (i + 1) / 2 + j, k * NV + i, k * NV + j, 0);
      }
      for (int l = 0; l < 16; ++l) {
        const int a = ANC[16 * k + l];
        if (a < 0) continue;
        t.w[W_BR + st * (NBSLOT + 1) + q / 16][16 * b + q % 16] = ldl_item(k * NV + a, k * NV + a, OFF_ONE, 0);
        ++q;
      }
      for (int l = 0; l < 16; ++l) t.w[W_BR + st * (NBSLOT + 1) + NBSLOT][16 * b + l] = (uint32_t)(k * NV + k);
    }
  // trunk pivot k: its pairs, then its row scalings, one item per lane
  for (int k = 0; k < NT; ++k) {
    for (int lane = 0; lane < 64; ++lane) t.w[W_TR + k][lane] = ldl_item(OFF_JUNK + lane, 0, 0, 0);
    int q = 0;
    for (int pp = LDL_START[k]; pp < LDL_START[k + 1]; ++pp, ++q)
      t.w[W_TR + k][q] = ldl_item(LDL_I[pp] * NV + LDL_J[pp], k * NV + LDL_I[pp], k * NV + LDL_J[pp], 1);
    for (int l = 0; l < 16; ++l)
      if (ANC[16 * k + l] >= 0) t.w[W_TR + k][q++] = ldl_item(k * NV + ANC[16 * k + l], k * NV + ANC[16 * k + l], OFF_ONE, 0);
  }
  // trunk entry (i, j) at lane i (i + 1) / 2 + j: its offset and the branch pivots below i
  for (int lane = 0; lane < 64; ++lane) t.w[W_TG][lane] = 0u;
  for (int i = 0, tp = 0; i < NT; ++i)
    for (int j = 0; j <= i; ++j, ++tp) {
      uint32_t m = 0;
      for (int k = NT; k < NV; ++k) m |= dof_is_anc(i, k) ? 1u << (k - NT) : 0u;
      t.w[W_TG][tp] = (uint32_t)(i * NV + j) | m << 16;
    }
  for (int b = 0; b < NB; ++b) {
    for (int i = 0; i < 4; ++i) t.quat[b][i] = BODY_QUAT[4 * b + i];
    for (int i = 0; i < 3; ++i) {
      t.pos[b][i] = BODY_POS[3 * b + i];
      t.ipos[b][i] = BODY_IPOS[3 * b + i];
    }
    for (int i = 0; i < 6; ++i) t.inertia[b][i] = BODY_INERTIA[6 * b + i];
    t.mass[b] = BODY_MASS[b];
    t.hinge0[b] = (uint8_t)BODY_HINGE0[b];
    t.nhinge[b] = (uint8_t)BODY_NHINGE[b];
  }
  for (int j = 0; j < NHINGE; ++j) {
    for (int i = 0; i < 3; ++i) {
      t.hax[j][i] = HINGE_AXIS[3 * j + i];
      t.hpos[j][i] = HINGE_POS[3 * j + i];
    }
    t.lo[j] = HINGE_LO[j];
    t.hi[j] = HINGE_HI[j];
    t.stiff[j] = HINGE_STIFF[j];
    t.damp[j] = HINGE_DAMP[j];
    t.arm[j] = HINGE_ARM[j];
  }
  for (int s = 0; s < NSPH; ++s) {
    for (int i = 0; i < 3; ++i) t.sph_pos[s][i] = SPHERE_POS[3 * s + i];
    t.sph_r[s] = SPHERE_R[s];
  }
  for (int i = 0; i < NV; ++i) t.act_of_dof[i] = (uint8_t)NONE;
  for (int k = 0; k < NACT; ++k) {
    t.gear[k] = ACT_GEAR[k];
    t.act_of_dof[ACT_DOF[k]] = (uint8_t)k;
  }
  return t;
}
__device__ constexpr Shared SHARED = make_shared();

// the block's copy of SHARED (one wave per block)
HM_INLINE void load_shared(Shared& S, int lane) {
  static_assert(sizeof(Shared) % 8 == 0, "Shared copies as doubles");
  const double* src = reinterpret_cast<const double*>(&SHARED);
  double* dst = reinterpret_cast<double*>(&S);
#pragma unroll 8
  for (int i = lane; i < (int)(sizeof(Shared) / 8); i += 64) dst[i] = src[i];
  WAVE_SYNC();
}

// a double broadcast from lane l (uniform) of the wave
HM_INLINE double read_lane(double v, int l) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// one env's working state (LDS, one wave)
struct Wave {
  double s[NQ + NV + NACT];  // qpos ++ qvel ++ ctrl
  double rot[NHINGE][9], Qloc[NB][9], oloc[NB][3], lax[NHINGE][3], lanc[NHINGE][3];
  double R[NB][9], xpos[NB][3], xipos[NB][3], haxis[NHINGE][3], hanchor[NHINGE][3], fsph[NSPH][6];
  // forward()'s outputs that accelerations() and the reward read, contiguous: the
  // kinematics cache (KCACHE doubles, com .. cfrc) a step leaves beside the env state
  double com[3], cinert[NB][10], cdof[NV][6], cdof_dot[NV][6], cvel[NB][6], cfrc[NB][6];
  double fb[NB][6], crb[NB][10];
  double F[NV][6];
  // L, then (contiguous, addressed as offsets from L: OFF_ONE, OFF_C, OFF_JUNK) the 1.0 of
  // the row scalings, the branch pivots' trunk products, and the target of lanes with no
  // entry (branch-free stores)
  double L[NV][NV], one, C[NCONTRIB], junk[64], x[NV];
  double red[2];
};
constexpr int KCACHE = 3 + NB * 10 + NV * 6 * 2 + NB * 6 * 2;
static_assert(offsetof(Wave, fb) - offsetof(Wave, com) == KCACHE * sizeof(double), "kinematics cache span");
// The kinematics cache of an env: what forward() computed from the state the step left
// (env_state's per-env tail, AoS: the wave's lanes read / write consecutive doubles).
// The next step starts from it instead of its first substep's forward() -- the same
// values, so bit-identical (every writer of a Humanoid env state writes its cache).
HM_INLINE void save_kcache(const Wave& W, double* dst, int lane) {
  const double* src = W.com;
#pragma unroll
  for (int i = 0; i < (KCACHE + 63) / 64; ++i)
    if (lane + 64 * i < KCACHE) dst[lane + 64 * i] = src[lane + 64 * i];
}
HM_INLINE void load_kcache(Wave& W, const double* src, int lane) {
  double* dst = W.com;
#pragma unroll
  for (int i = 0; i < (KCACHE + 63) / 64; ++i)
    if (lane + 64 * i < KCACHE) dst[lane + 64 * i] = src[lane + 64 * i];
}
static_assert(offsetof(Wave, one) - offsetof(Wave, L) == OFF_ONE * sizeof(double) &&
                  offsetof(Wave, C) - offsetof(Wave, L) == OFF_C * sizeof(double) &&
                  offsetof(Wave, junk) - offsetof(Wave, L) == OFF_JUNK * sizeof(double),
              "W.L offsets of the L^T D L items");

HM_INLINE int path_body(uint32_t p0, uint32_t p1, int s) { return (int)byte_of(s < 4 ? p0 : p1, s & 3); }

// kinematics, com-based inertias / axes / velocities and contact forces of W.s.  The
// chains down the tree (world poses, velocities) run per body along its own path from
// the root -- every lane repeats its ancestors' arithmetic exactly, so no level needs
// a round trip through LDS.
HM_INLINE void forward(Wave& W, const Shared& S, int lane, int64_t* st = nullptr) {
  const double* q = W.s;
  const double* qd = W.s + NQ;
  // hinge rotations (all hinges at once) and the root's orientation
  if (lane >= 32 && lane < 32 + NHINGE) {
    const int j = lane - 32;
    double sn, cs;
    sincos(q[7 + j], &sn, &cs);
    axis_rot(S.hax[j], sn, cs, W.rot[j]);
  } else if (lane == 0) {
    const double qn = sqrt(((q[3] * q[3] + q[4] * q[4]) + q[5] * q[5]) + q[6] * q[6]);
    quat_mat(q[3] / qn, q[4] / qn, q[5] / qn, q[6] / qn, W.R[0]);
    W.xpos[0][0] = q[0];
    W.xpos[0][1] = q[1];
    W.xpos[0][2] = q[2];
  }
  WAVE_SYNC();
  // each body's pose in its parent's frame (after its hinges), one lane per (body b, row
  // r): every product here takes row r of the body's running rotation Q times constant /
  // LDS matrices and vectors, so a row's lane carries the row through the same operations
  // (mm3 / mv3 row r) as a body-per-lane loop over all three
  {
    const int b = lane & 15, r = lane >> 4;
    if (b >= 1 && b < NB && r < 3) {
      double Q[3], o;
      {
        double Qf[9];
        quat_mat(S.quat[b][0], S.quat[b][1], S.quat[b][2], S.quat[b][3], Qf);
#pragma unroll
        for (int c = 0; c < 3; ++c) Q[c] = r == 0 ? Qf[c] : (r == 1 ? Qf[3 + c] : Qf[6 + c]);
      }
      o = S.pos[b][r];
      const int h0 = S.hinge0[b], nh = S.nhinge[b];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (c < nh) {
          const int j = h0 + c;
          const double* hp = S.hpos[j];
          const double* hx = S.hax[j];
          const double* rt = W.rot[j];
          const double ra = (Q[0] * hp[0] + Q[1] * hp[1]) + Q[2] * hp[2];
          const double la = o + ra;
          W.lanc[j][r] = la;
          W.lax[j][r] = (Q[0] * hx[0] + Q[1] * hx[1]) + Q[2] * hx[2];
          double Qn[3];
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) Qn[jj] = (Q[0] * rt[jj] + Q[1] * rt[3 + jj]) + Q[2] * rt[6 + jj];
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) Q[jj] = Qn[jj];
          const double rb = (Q[0] * hp[0] + Q[1] * hp[1]) + Q[2] * hp[2];
          o = la - rb;
        }
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) W.Qloc[b][3 * r + c] = Q[c];
      W.oloc[b][r] = o;
    }
  }
  WAVE_SYNC();
  HM_STAMP(1);
  // world poses: body b composes its path from the root, one lane per (body b, row r):
  // row r of R Qloc and of R oloc need row r of R only
  {
    const int b = lane & 15, r = lane >> 4;
    if (b >= 1 && b < NB && r < 3) {
      const uint32_t p0 = S.w[W_PATH][b], p1 = S.w[W_PATH + 1][b];
      double R[3], x;
#pragma unroll
      for (int c = 0; c < 3; ++c) R[c] = W.R[0][3 * r + c];
      x = W.xpos[0][r];
#pragma unroll
      for (int s = 0; s < PATH_LEN; ++s) {
        const int a = path_body(p0, p1, s);
        const bool has = a != (int)NONE;
        const int ac = has ? a : 0;
        const double* Ql = W.Qloc[ac];
        const double* ol = W.oloc[ac];
        double Rn[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) Rn[c] = (R[0] * Ql[c] + R[1] * Ql[3 + c]) + R[2] * Ql[6 + c];
        const double off = (R[0] * ol[0] + R[1] * ol[1]) + R[2] * ol[2];
        x = has ? x + off : x;
#pragma unroll
        for (int c = 0; c < 3; ++c) R[c] = has ? Rn[c] : R[c];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) W.R[b][3 * r + c] = R[c];
      W.xpos[b][r] = x;
    }
  }
  WAVE_SYNC();
  HM_STAMP(2);
  // inertia centres (bodies) and hinge axes / anchors in the world (hinges)
  if (lane < NB) {
    double ri[3];
    mv3(W.R[lane], S.ipos[lane], ri);
#pragma unroll
    for (int i = 0; i < 3; ++i) W.xipos[lane][i] = W.xpos[lane][i] + ri[i];
  } else if (lane >= 32 && lane < 32 + NHINGE) {
    const int j = lane - 32;
    const int p = (int)byte_of(S.w[W_MISC][lane], 2);
    double ra[3];
    mv3(W.R[p], W.lax[j], W.haxis[j]);
    mv3(W.R[p], W.lanc[j], ra);
#pragma unroll
    for (int i = 0; i < 3; ++i) W.hanchor[j][i] = W.xpos[p][i] + ra[i];
  }
  WAVE_SYNC();
  if (lane < 3) {
    double acc = 0.0;
    for (int b = 0; b < NB; ++b) acc = acc + S.mass[b] * W.xipos[b][lane];
    W.com[lane] = acc / TOTAL_MASS;
  }
  WAVE_SYNC();
  {  // cinert, one lane per (body b, row r): row r of T = R Ib and of Iw = T R^T, and the
     // cinert entries on that row of Iw (the same expressions as a body-per-lane mm3 pair)
    const int b = lane & 15, r = lane >> 4;
    if (b < NB && r < 3) {
      const double* I6 = S.inertia[b];
      const double Ib[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
      const double* R = W.R[b];
      double T[3], Iw[3], d[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) T[j] = (R[3 * r] * Ib[j] + R[3 * r + 1] * Ib[3 + j]) + R[3 * r + 2] * Ib[6 + j];
#pragma unroll
      for (int j = 0; j < 3; ++j) Iw[j] = (T[0] * R[3 * j] + T[1] * R[3 * j + 1]) + T[2] * R[3 * j + 2];
      const double m = S.mass[b];
#pragma unroll
      for (int i = 0; i < 3; ++i) d[i] = W.xipos[b][i] - W.com[i];
      double* ci = W.cinert[b];
      if (r == 0) {
        ci[0] = Iw[0] + m * (d[1] * d[1] + d[2] * d[2]);
        ci[3] = Iw[1] - m * (d[0] * d[1]);
        ci[4] = Iw[2] - m * (d[0] * d[2]);
      } else if (r == 1) {
        ci[1] = Iw[1] + m * (d[0] * d[0] + d[2] * d[2]);
        ci[5] = Iw[2] - m * (d[1] * d[2]);
      } else {
        ci[2] = Iw[2] + m * (d[0] * d[0] + d[1] * d[1]);
        ci[6] = m * d[0];
        ci[7] = m * d[1];
        ci[8] = m * d[2];
        ci[9] = m;
      }
    }
  }
  if (lane >= 32 && lane < 32 + NV) {  // cdof
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
  HM_STAMP(3);
  // cvel and cdof_dot (MuJoCo mj_comVel order).  The velocity walk down body b's path is
  // element-wise (cv += cdof qd), so one lane per (body b, element pair ep) carries two of
  // its six elements; the walk leaves the velocity in front of each of the body's own
  // hinges in scratch (W.L, free until the mass matrix), and then one lane per (body,
  // own hinge) forms that hinge's cdof_dot = cv x cdof -- the same operations per element
  // as a body-per-lane walk that crosses every dof of its path and keeps its own
  {
    double* const X = &W.L[0][0];  // [NB][3][6] cv in front of own hinge c; [234..240) cv after the root's translation
    const int b = lane & 15, ep = lane >> 4;
    if (b < NB && ep < 3) {
      double cv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = 2 * ep + i;
        cv[i] = 0.0 + ((W.cdof[0][e] * qd[0] + W.cdof[1][e] * qd[1]) + W.cdof[2][e] * qd[2]);
        if (b == 0) X[NB * 18 + e] = cv[i];
        cv[i] = cv[i] + ((W.cdof[3][e] * qd[3] + W.cdof[4][e] * qd[4]) + W.cdof[5][e] * qd[5]);
      }
      uint32_t pw[PD_WORDS];
#pragma unroll
      for (int q = 0; q < PD_WORDS; ++q) pw[q] = S.w[W_PDOF + q][lane];
#pragma unroll
      for (int t = 0; t < MAXPD; ++t) {  // the path's hinge dofs in order (W_PDOF)
        const uint32_t pb = byte_of(pw[t >> 2], t & 3);
        const bool has = (pb & 31u) != 31u;
        const int d = has ? (int)(pb & 31u) : 6;
        const double qdd = qd[d];
        if (has && (pb & 0x20u)) {  // own hinge c: the velocity in front of it
          const int c = (int)(pb >> 6);
          X[(b * 3 + c) * 6 + 2 * ep] = cv[0];
          X[(b * 3 + c) * 6 + 2 * ep + 1] = cv[1];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) cv[i] = has ? cv[i] + W.cdof[d][2 * ep + i] * qdd : cv[i];
      }
      W.cvel[b][2 * ep] = cv[0];
      W.cvel[b][2 * ep + 1] = cv[1];
    }
    WAVE_SYNC();
    // lane (b, c < 3): own hinge c of body b; lanes 48..50: the root's rotational dofs
    // 3..5 (from the velocity after its translation); lanes 51..53: dofs 0..2 (zero)
    const int c = lane >> 4;
    if (c < 3) {
      if (b < NB && c < (int)S.nhinge[b]) {
        const int d = 6 + S.hinge0[b] + c;
        cross_motion(X + (b * 3 + c) * 6, W.cdof[d], W.cdof_dot[d]);
      }
    } else if (b < 3) {
      cross_motion(X + NB * 18, W.cdof[3 + b], W.cdof_dot[3 + b]);
    } else if (b < 6) {
#pragma unroll
      for (int i = 0; i < 6; ++i) W.cdof_dot[b - 3][i] = 0.0;
    }
  }
  WAVE_SYNC();
  HM_STAMP(4);
  // ground contact: sphere s of body b against z = 0, at the sphere's lowest point
  if (lane < NSPH) {
    const int s = lane;
    const int b = (int)byte_of(S.w[W_MISC][lane], 1);
    const double r = S.sph_r[s];
    double cs[3], c[3], rel[3], wr[3], v[3], fv[3];
    mv3(W.R[b], S.sph_pos[s], cs);
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
    const uint32_t own = S.w[W_OWN][lane];
    const int s0 = (int)byte_of(own, 2), ns = (int)byte_of(own, 3);
    for (int s = s0; s < s0 + ns; ++s)
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[i] = acc[i] + W.fsph[s][i];
#pragma unroll
    for (int i = 0; i < 6; ++i) W.cfrc[b][i] = acc[i];
  }
  WAVE_SYNC();
  HM_STAMP(5);
}

__device__ inline double clamp_ctrl(double c) { return c < -CTRL_LIMIT ? -CTRL_LIMIT : (c > CTRL_LIMIT ? CTRL_LIMIT : c); }

// gear * clip(ctrl) at dof i (0 for the unactuated root dofs)
HM_INLINE double actuator_force(const Shared& S, const double* ctrl, int i) {
  const int k = S.act_of_dof[i];
  return k == (int)NONE ? 0.0 : S.gear[k] * clamp_ctrl(ctrl[k]);
}

// W.x <- qdd of M qdd = qfrc_actuator + passive + limits - (bias - contact); needs forward(W)
HM_INLINE void accelerations(Wave& W, const Shared& S, int lane, int64_t* st = nullptr) {
  const double* q = W.s;
  const double* qd = W.s + NQ;
  const double* ctrl = W.s + NQ + NV;
  // cacc along body b's path, one lane per (body b, element pair ep): the path walk's
  // multiply-adds are element-wise, so each lane carries two of the six elements through
  // the same operation sequence (a third of the body-per-lane walk's instructions); the
  // pairs meet in W.F (free until the F phase) for the bias force on body lanes
  {
    const int b = lane & 15, ep = lane >> 4;
    if (b < NB && ep < 3) {
      double ca[2] = {0.0, ep == 2 ? 0.0 + GRAV : 0.0};
#pragma unroll
      for (int k = 3; k < 6; ++k)
#pragma unroll
        for (int i = 0; i < 2; ++i) ca[i] = ca[i] + W.cdof_dot[k][2 * ep + i] * qd[k];
      uint32_t pw[PD_WORDS];
#pragma unroll
      for (int q = 0; q < PD_WORDS; ++q) pw[q] = S.w[W_PDOF + q][lane];
#pragma unroll
      for (int t = 0; t < MAXPD; ++t) {  // the path's hinge dofs in order (W_PDOF)
        const uint32_t pb = byte_of(pw[t >> 2], t & 3);
        const bool has = (pb & 31u) != 31u;
        const int d = has ? (int)(pb & 31u) : 6;
        const double qdd = qd[d];
#pragma unroll
        for (int i = 0; i < 2; ++i) ca[i] = has ? ca[i] + W.cdof_dot[d][2 * ep + i] * qdd : ca[i];
      }
      W.F[b][2 * ep] = ca[0];
      W.F[b][2 * ep + 1] = ca[1];
    }
  }
  WAVE_SYNC();
  // the bias force of body `lane` (RNEA forward pass)
  if (lane < NB) {
    const int b = lane;
    double ca[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) ca[i] = W.F[b][i];
    double Ia[6], Iv[6], cf[6];
    mul_inert(W.cinert[b], ca, Ia);
    mul_inert(W.cinert[b], W.cvel[b], Iv);
    cross_force(W.cvel[b], Iv, cf);
#pragma unroll
    for (int i = 0; i < 6; ++i) W.fb[b][i] = (Ia[i] + cf[i]) - W.cfrc[b][i];
#pragma unroll
    for (int i = 0; i < 10; ++i) W.crb[b][i] = W.cinert[b][i];
  }
  WAVE_SYNC();
  HM_STAMP(6);
  // subtree sums, leaves -> root: a parent adds its children in descending index.  One
  // lane per (parent slot, element): a level's (at most four) parents x the 16 elements
  // of fb (6) ++ crb (10) fill the wave, so each lane adds its element's three child
  // values -- the same adds in the same order per element as a parent-per-lane loop over
  // all 16, at a sixteenth of the instructions (subtree phase 10.6 k -> see DESIGN §3b)
  {
    const int slot = lane >> 4, el = lane & 15;
    double* const eb = el < 6 ? &W.fb[0][el] : &W.crb[0][el - 6];  // element el of body 0
    const int es = el < 6 ? 6 : 10;                                 // its stride over bodies
#pragma unroll 1
    for (int lv = NLEVEL - 2; lv >= 0; --lv) {
      const uint32_t ts = S.w[W_SUB + lv][slot];
      const int p = (int)byte_of(ts, 0);
      if (p != (int)NONE) {
        // every child slot loads (a missing child reads the parent) so the loads batch;
        // only existing children add
        double v = eb[p * es], cv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int ch = (int)byte_of(ts, k + 1);
          cv[k] = eb[(ch == (int)NONE ? p : ch) * es];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) v = byte_of(ts, k + 1) != NONE ? v + cv[k] : v;
        eb[p * es] = v;
      }
      WAVE_SYNC();
    }
  }
  HM_STAMP(7);
  // per dof i: F_i = crb(body(i)) cdof_i and the generalised force
  if (lane < NV) {
    const int i = lane;
    const int bi = (int)byte_of(S.w[W_MISC][lane], 0);
    mul_inert(W.crb[bi], W.cdof[i], W.F[i]);
    const double bias = dot6(W.cdof[i], W.fb[bi]);
    double t = actuator_force(S, ctrl, i) - bias;
    if (i >= 6) {
      const int j = i - 6;
      const double qj = q[7 + j], vj = qd[i];
      const double lo = S.lo[j], hi = S.hi[j];
      const double lim = qj < lo ? KL * (lo - qj) - CL * vj : (qj > hi ? KL * (hi - qj) - CL * vj : 0.0);
      const double passive = (-(S.stiff[j] * qj) - S.damp[j] * vj) + lim;
      t = t + passive;
    }
    W.x[i] = t;
  }
  WAVE_SYNC();
  HM_STAMP(8);
  // mass-matrix entries M_ij = cdof_j . F_i (j = i or an ancestor), all lanes at once
  double* Lf = &W.L[0][0];
  const int junk = OFF_JUNK + lane;  // W.junk[lane]
#pragma unroll
  for (int r = 0; r < 2 * N_ENT_WORDS; ++r) {
    const uint32_t e = (S.w[W_ENT + (r >> 1)][lane] >> (16 * (r & 1))) & 0xffffu;
    const int i = (int)(e & 0xff), j = (int)((e >> 8) & 0xff);
    const int ic = i == (int)NONE ? 0 : i, jc = j == (int)NONE ? 0 : j;
    const double v = dot6(W.cdof[jc], W.F[ic]);
    Lf[i == (int)NONE ? junk : ic * NV + jc] = v;
  }
  WAVE_SYNC();
  if (lane >= 6 && lane < NV) W.L[lane][lane] = W.L[lane][lane] + S.arm[lane - 6];
  WAVE_SYNC();
  HM_STAMP(9);
  // L^T D L, leaves first (the branch-parallel schedule above).  Branch steps: each lane
  // reads its items' operands and its pivot's diagonal, then writes (reads before writes:
  // one phase per step)
  if (lane == 0) W.one = 1.0;
  WAVE_SYNC();
#pragma unroll 1
  for (int st = 0; st < NBSTEP; ++st) {
    uint32_t it[NBSLOT];
#pragma unroll
    for (int q = 0; q < NBSLOT; ++q) it[q] = S.w[W_BR + st * (NBSLOT + 1) + q][lane];
    const double lkk = Lf[S.w[W_BR + st * (NBSLOT + 1) + NBSLOT][lane]];
    double vd[NBSLOT], v1[NBSLOT], v2[NBSLOT];
#pragma unroll
    for (int q = 0; q < NBSLOT; ++q) {
      vd[q] = Lf[it[q] & 0x7ffu];
      v1[q] = Lf[(it[q] >> 11) & 0x3ffu];
      v2[q] = Lf[(it[q] >> 21) & 0x3ffu];
    }
    const double invd = 1.0 / lkk;
#pragma unroll
    for (int q = 0; q < NBSLOT; ++q) {
      const double p = v1[q] * (v2[q] * invd);
      Lf[it[q] & 0x7ffu] = (it[q] >> 31) ? vd[q] - p : p;
    }
    WAVE_SYNC();
  }
  // trunk gather: entry (i, j) minus the branch pivots' products, in descending pivot order
  if (lane < NTP) {
    const uint32_t tg = S.w[W_TG][lane];
    const int off = (int)(tg & 0xffffu);
    const uint32_t m = tg >> 16;
    double v = Lf[off], c[NV - NT];
#pragma unroll
    for (int q = 0; q < NV - NT; ++q) c[q] = Lf[OFF_C + q * NTP + lane];
#pragma unroll
    for (int q = NV - NT - 1; q >= 0; --q) v = ((m >> q) & 1u) ? v - c[q] : v;
    Lf[off] = v;
  }
  WAVE_SYNC();
  // trunk pivots in sequence, one item per lane (W_TR): pivot k updates every (ancestor i,
  // ancestor-or-self j of i) pair from its still unscaled row, then scales its row (reads
  // before writes: one phase per pivot).  The next pivot's reciprocal diagonal is formed
  // from the value pivot k just computed for (k - 1, k - 1) -- its final value, pivot k
  // being the last to update it -- on the lane that holds it, while the next pivot's LDS
  // operands are in flight, and broadcast by readlane: the division leaves the chain.
  uint32_t it = S.w[W_TR + NT - 1][lane];
  double invd = 1.0 / Lf[(NT - 1) * NV + NT - 1];
  double vd = Lf[it & 0x7ffu], v1 = Lf[(it >> 11) & 0x3ffu], v2 = Lf[(it >> 21) & 0x3ffu];
#pragma unroll 1
  for (int k = NT - 1; k >= 0; --k) {
    const uint32_t cur = it;
    const double p = v1 * (v2 * invd);
    const double r = (cur >> 31) ? vd - p : p;
    Lf[cur & 0x7ffu] = r;
    if (k > 0) {
      WAVE_SYNC();
      it = S.w[W_TR + k - 1][lane];
      vd = Lf[it & 0x7ffu];
      v1 = Lf[(it >> 11) & 0x3ffu];
      v2 = Lf[(it >> 21) & 0x3ffu];
      invd = read_lane(1.0 / r, (int)((TRUNK_DIAG_LANES >> (6 * k)) & 63u));
    }
  }
  WAVE_SYNC();
  HM_STAMP(10);
  // the solves with x in registers (lane j holds x_j), the pivot broadcast by readlane:
  // L^T y = x (leaves first), D z = y, L x = z (column by column)
  double x = lane < NV ? W.x[lane] : 0.0;
  const int lr = lane < NV ? lane : 0;
#pragma unroll 4
  for (int i = NV - 1; i >= 0; --i) {
    const double xi = read_lane(x, i);
    const double y = x - W.L[i][lr] * xi;
    x = ((MASKS.anc[i] >> lane) & 1u) ? y : x;
  }
  if (lane < NV) x = x / W.L[lane][lane];
#pragma unroll 4
  for (int j = 0; j < NV; ++j) {
    const double xj = read_lane(x, j);
    const double y = x - W.L[lr][j] * xj;
    x = ((MASKS.desc[j] >> lane) & 1u) ? y : x;
  }
  if (lane < NV) W.x[lane] = x;
  WAVE_SYNC();
  HM_STAMP(11);
}

// semi-implicit Euler over dt in place on W.s from the accelerations in W.x
HM_INLINE void integrate(Wave& W, int lane) {
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
}

// one dt in place on W.s; returns the COM x of the state it started from
HM_INLINE double substep(Wave& W, const Shared& S, int lane) {
  forward(W, S, lane);
  const double com_x = W.com[0];
  accelerations(W, S, lane);
  integrate(W, lane);
  return com_x;
}

// reward and done of a step that started at COM x x_before; needs forward(W) of the
// new state.  reward = 0.25 dx_com / dt + 5 - 0.1 |ctrl|^2 - min(0.5e-6 |cfrc_ext|^2, 10)
HM_INLINE void reward_done(Wave& W, int lane, double x_before, double& rew, bool& done) {
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
__device__ inline void observation(const Wave& W, const Shared& S, int lane, Out out) {
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
      v = actuator_force(S, W.s + NQ + NV, k - 269);
    } else {
      const int b = (k - 292) / 6 - 1, c = (k - 292) % 6;
      v = b < 0 ? 0.0 : W.cfrc[b][c];
    }
    out(k, v);
  }
}

}  // namespace hm

constexpr int HM_NQ = hm::NQ, HM_NV = hm::NV, HM_ACT = hm::NACT, HM_NS = hm::NS, HM_OBS = hm::OBS, HM_NU = hm::NU;
constexpr int HM_KCACHE = hm::KCACHE;

}  // namespace mrl
