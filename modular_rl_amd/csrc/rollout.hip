// Batched lock-step rollout: E envs per GPU advance one step per launch.
//
// Replaces the reference's serial per-step loop (core.py:182-221):
//     ob = agent.obfilt(ob)                 ZFilter, filters.py:30-38
//     action, {"prob"} = agent.act(ob)      StochPolicy.act, core.py:261-267
//     ob, rew, done, _ = env.step(action)   gym
//     agent.rewfilt(rew)                    stats only, core.py:198-199
// Per launch (step t) every block
//   1. merges the per-block Welford partials of the E raw observations of step t
//      (and rewards of step t-1) -- published by launch t-1 -- into the running
//      stat (every block derives the identical state; block 0 stores it; ping-pong
//      buffers by step parity),
//   2. normalises its envs' observations (x - mean)/(std + 1e-8), clip +-5, stores
//      them as the trajectory rows (fp32) and in LDS,
//   3. runs the policy MLP forward on MFMA (32 envs per wave, image in LDS),
//   4. samples the action (Philox counter stream or injected noise),
//   5. steps the env (fp64), auto-resets finished episodes, writes reward/flags,
//   6. publishes the block's Welford partial of the new raw obs and the reward.
// Kernels are templated on the env so every per-env array has a compile-time size
// (registers, no scratch).
#include <math.h>

#include <type_traits>

#include "../../include/mrl_hip.h"
#include "envs.h"
#include "mlp_device.h"

namespace mrl {

constexpr int RB = 256;  // threads per block
constexpr int ENVS_PER_BLOCK = 64;  // fused step: 4 waves x 16 envs
constexpr int MAXD = 16;  // obs dims + 1 (reward)

// Hopper-v2 in the fused step kernel, where the four 16-lane rows of a wave hold
// the SAME 16 envs: row g evaluates sincos of segment angle g and the contacts of
// capsule g, and the rows exchange the results, so every row continues with the
// identical state.  All lanes must be active.
// the persistent kernel's capsule constants: 2 -- the row's own six, read from the LDS
// table once per launch and held in registers; 1 -- read from the LDS table every substep;
// 0 -- per-substep selects (A/B builds)
#ifndef MRL_HP_CAP_LDS
#define MRL_HP_CAP_LDS 2
#endif
struct HopperQuad {
  int g;
  const double* capc;  // mode 2: the row's capsule {rad, mu, u0, u1, w0, w1}; mode 1: HP_CAP
                       // in LDS ([field][k]); or null
  __device__ CapsuleC capsule(int) const {
    if (MRL_HP_CAP_LDS == 2 && capc != nullptr) return CapsuleC{capc[0], capc[1], capc[2], capc[3], capc[4], capc[5]};
    if (MRL_HP_CAP_LDS == 1 && capc != nullptr)
      return CapsuleC{capc[g], capc[4 + g], capc[8 + g], capc[12 + g], capc[16 + g], capc[20 + g]};
    return capsule_const(g);
  }
  __device__ void sincos4(const double* phi, double* s, double* c, double& so, double& co) const {
    double sx, cx;
    sincos(sel4(g, phi[0], phi[1], phi[2], phi[3]), &sx, &cx);
    quads(sx, s);
    quads(cx, c);
    so = sx;
    co = cx;
  }
  // segment k == g's value: the row's own (sel4(g, quads(x)) is x, bit for bit), with no
  // wait for the row exchange and no select
  __device__ double own(int, const double*, double v) const { return v; }
  template <class F>
  __device__ void contacts(F f, double (*ct)[3]) const {
    double own[3], x[4];
    f(g, own);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      quads(own[i], x);
#pragma unroll
      for (int k = 0; k < 4; ++k) ct[k][i] = x[k];
    }
  }
};

template <int ENV>
struct EnvC;
template <>
struct EnvC<MRL_ENV_CARTPOLE> {
  static constexpr int NS = CP_NS, OBS = CP_OBS, ACT = 2, DISCRETE = 1, MAX_STEPS = 200, NU = 4, OBS_SLOTS = 0;
  __device__ static void reset(const double* u, double* s) { cartpole_reset(u, s); }
  __device__ static void obs(const double* s, double* o) { cartpole_obs(s, o); }
  __device__ static void step_disc(double* s, int a, double& rew, bool& done) { cartpole_step(s, a, rew, done); }
  __device__ static void step_cont(double*, const float*, double&, bool&) {}
  __device__ static void step_cont_quad(double*, const float*, double&, bool&, int, const double*) {}
  template <class Out>
  __device__ static void obs_out(const double* s, Out out) {
    double o[OBS];
    cartpole_obs(s, o);
#pragma unroll
    for (int k = 0; k < OBS; ++k) out(k, o[k]);
  }
};
template <>
struct EnvC<MRL_ENV_HOPPER> {
  static constexpr int NS = HP_NS, OBS = HP_OBS, ACT = HP_ACT, DISCRETE = 0, MAX_STEPS = 1000, NU = 12,
                       OBS_SLOTS = 0;
  __device__ static void reset(const double* u, double* s) { hopper_reset(u, s); }
  __device__ static void obs(const double* s, double* o) { hopper_obs(s, o); }
  __device__ static void step_disc(double*, int, double&, bool&) {}
  __device__ static void step_cont(double* s, const float* a, double& rew, bool& done) { hopper_step(s, a, rew, done); }
  __device__ static void step_cont_quad(double* s, const float* a, double& rew, bool& done, int g,
                                        const double* capc) {
    hopper_step(s, a, rew, done, HopperQuad{g, capc});
  }
  template <class Out>
  __device__ static void obs_out(const double* s, Out out) {
    double o[OBS];
    hopper_obs(s, o);
#pragma unroll
    for (int k = 0; k < OBS; ++k) out(k, o[k]);
  }
};
template <>
struct EnvC<MRL_ENV_HUMANOID> {  // stepped by the wave-per-env kernels (hm_*_kernel), not per thread
  static constexpr int NS = HM_NS, OBS = HM_OBS, ACT = HM_ACT, DISCRETE = 0, MAX_STEPS = 1000, NU = HM_NU,
                       OBS_SLOTS = 0;
  __device__ static void reset(const double*, double*) {}
  __device__ static void step_disc(double*, int, double&, bool&) {}
  __device__ static void step_cont(double*, const float*, double&, bool&) {}
  template <class Out>
  __device__ static void obs_out(const double*, Out) {}
};

struct EnvInfo {
  int ns, obs, act, discrete, max_steps;
};
__host__ __device__ inline EnvInfo env_info(int id) {
  if (id == MRL_ENV_CARTPOLE) return EnvInfo{CP_NS, CP_OBS, 2, 1, 200};
  if (id == MRL_ENV_HUMANOID) return EnvInfo{HM_NS, HM_OBS, HM_ACT, 0, 1000};
  return EnvInfo{HP_NS, HP_OBS, HP_ACT, 0, 1000};
}
__host__ __device__ inline int filt_doubles(int obs) { return 2 + 2 * (obs + 1); }

struct RollArgs {
  mrl_rollout_desc d;
  mrl_rollout_bufs b;
  int nb;      // blocks
  int FS, RS;  // filter / record doubles
};

// reset-noise uniforms for one env: (gid, episode counter) on domain 1
// ------------------------------------------------------------------ rollout policy forward
// One wave = 16 envs on v_mfma_f32_16x16x4_f32 (mlp_layout.h, rollout image): the
// step kernel is a latency chain at one wave per SIMD, and 16-row tiles halve both
// the MFMA chain and the tanh work of a 32-row tile.  The weight fragments of the
// wave go straight from global memory (L2-resident rollout image) into registers,
// loaded at kernel entry so their latency hides under the filter merge.
template <int O, int A>
struct RWeights {
  static constexpr RDims R = rollout_dims(O);
  float4 a0[4][R.KS0p / 4];
  const bf16x8* w1s = nullptr;  // the split W1 fragments (image section bs1), staged in LDS
  float4 b0[4], b1[4];
  float4 hv[A][4];
  float hb[A];
  __device__ void load(const float* __restrict__ img, int lane) {
    const int g = lane >> 4;
    const float4* f = reinterpret_cast<const float4*>(img);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo)
#pragma unroll
      for (int s4 = 0; s4 < R.KS0p / 4; ++s4) a0[mo][s4] = f[(R.a0 >> 2) + (mo * (R.KS0p / 4) + s4) * 64 + lane];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      b0[mt] = f[(R.b0 >> 2) + g * 4 + mt];
      b1[mt] = f[(R.b1 >> 2) + g * 4 + mt];
    }
#pragma unroll
    for (int o = 0; o < A; ++o)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) hv[o][mt] = f[(R.hv >> 2) + (g * MAX_OUT + o) * 4 + mt];
#pragma unroll
    for (int o = 0; o < A; ++o) hb[o] = img[R.hb + o];
  }
};

// bf16 compute mode: layer-0 / layer-1 fragments of v_mfma_f32_16x16x32_bf16 (image
// segments ba0 / ba1), biases and the VALU head as in RWeights
template <int O, int A>
struct RWeightsB {
  static constexpr RDims R = rollout_dims(O);
  bf16x8 a0[4];
  bf16x8 a1[4][2];
  float4 b0[4], b1[4];
  float4 hv[A][4];
  float hb[A];
  __device__ void load(const float* __restrict__ img, int lane) {
    const int g = lane >> 4;
    const bf16x8* f0 = reinterpret_cast<const bf16x8*>(img + R.ba0);
    const bf16x8* f1 = reinterpret_cast<const bf16x8*>(img + R.ba1);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      a0[mo] = f0[mo * 64 + lane];
#pragma unroll
      for (int p = 0; p < 2; ++p) a1[mo][p] = f1[(mo * 2 + p) * 64 + lane];
    }
    const float4* f = reinterpret_cast<const float4*>(img);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      b0[mt] = f[(R.b0 >> 2) + g * 4 + mt];
      b1[mt] = f[(R.b1 >> 2) + g * 4 + mt];
    }
#pragma unroll
    for (int o = 0; o < A; ++o)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) hv[o][mt] = f[(R.hv >> 2) + (g * MAX_OUT + o) * 4 + mt];
#pragma unroll
    for (int o = 0; o < A; ++o) hb[o] = img[R.hb + o];
  }
};

template <int O, int A, bool BF>
using RollWeights = typename std::conditional<BF, RWeightsB<O, A>, RWeights<O, A>>::type;

__device__ inline f32x4 as_f32x4(float4 v) {
  f32x4 r;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
  r[3] = v.w;
  return r;
}

__device__ inline void tanh4(f32x4& a) {
#pragma unroll
  for (int r = 0; r < 4; ++r) a[r] = tanh_fast(a[r]);
}

// bf16 RNE round trip (the bf16 compute mode's operand rounding on the f32-input MFMA)
__device__ inline float bf16r(float x) { return (float)(__bf16)x; }
template <bool BF>
__device__ inline void tanh4r(f32x4& a) {
#ifdef MRL_ABL_NOTANH  // diagnostic timing build only (results are wrong)
  return;
#endif
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const f32x2 t = tanh_fast2(f32x2{a[r], a[r + 1]});
    a[r] = BF ? bf16r(t.x) : t.x;
    a[r + 1] = BF ? bf16r(t.y) : t.y;
  }
}

// head rows z[o] of the wave's 16 envs (every lane of an env's column ends with all A).
// BF (MRL_COMPUTE_BF16): x, h1, h2 rounded to bf16 (W0, W1 are rounded in the image),
// the operands mlp_rows_bf16 multiplies -- the products and sums stay f32, so the prob
// rows equal the update's bf16 forward up to f32 summation order.
#ifndef MRL_FWD_WPF  // 1: a k-step's twelve split W1 fragments read from LDS ahead of its MFMAs
#define MRL_FWD_WPF 1
#endif
template <int O, int A, bool BF, class XL>
__device__ inline void forward16(const RWeights<O, A>& w, const XL& xl, int lane, float* z, int64_t* st = nullptr) {
  constexpr RDims R = RWeights<O, A>::R;
  const int g = lane >> 4;
  // the split W1 fragments of k-step s, [tile mo][part p]: k-step 0's issued before layer 0,
  // k-step 1's once k-step 0's MFMAs are issued -- each lands under other work instead of
  // an LDS round trip in front of every MFMA group (the persistent kernel's registers are
  // held by the fp64 dynamics, not here)
  bf16x8 wf[4][3];
  auto load_wf = [&](int s) {
#pragma unroll
    for (int mo = 0; mo < 4; ++mo)
#pragma unroll
      for (int p = 0; p < 3; ++p) wf[mo][p] = w.w1s[(p * 8 + mo * 2 + s) * 64 + lane];
  };
  if (MRL_FWD_WPF) load_wf(0);
  float xb[R.KS0p];
#pragma unroll
  for (int ks = 0; ks < R.KS0p; ++ks) xb[ks] = ks < R.KS0 ? (BF ? bf16r(xl(4 * ks + g)) : xl(4 * ks + g)) : 0.f;
  f32x4 h1[4], h2[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    h1[m] = as_f32x4(w.b0[m]);
    h2[m] = as_f32x4(w.b1[m]);
  }
  // layer 0: four independent 16-unit accumulators
#pragma unroll
  for (int ks = 0; ks < R.KS0; ++ks)
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) h1[mo] = MFMA16(f4get(w.a0[mo][ks >> 2], ks & 3), xb[ks], h1[mo]);
  if (st != nullptr) st[9] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // layer 1 on split operands (fp32-accurate: h1 and W1 split exactly into three bf16
  // parts, six part products on v_mfma_f32_16x16x32_bf16, f32 accumulation): k-step s
  // covers tiles 2s, 2s+1 -- the lane's own registers, unit rb_unit(s, g, e) for element e
  // -- against the W1 fragments the rollout image holds split (section bs1)
  tanh4r<BF>(h1[0]);
  tanh4r<BF>(h1[1]);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 hp[3];
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      bf16x2 a, c, e, a2, c2, e2;
      split2(f32x2{h1[2 * s][r], h1[2 * s][r + 1]}, a, c, e);
      split2(f32x2{h1[2 * s + 1][r], h1[2 * s + 1][r + 1]}, a2, c2, e2);
      hp[0][r] = a[0]; hp[0][r + 1] = a[1]; hp[0][4 + r] = a2[0]; hp[0][4 + r + 1] = a2[1];
      hp[1][r] = c[0]; hp[1][r + 1] = c[1]; hp[1][4 + r] = c2[0]; hp[1][4 + r + 1] = c2[1];
      hp[2][r] = e[0]; hp[2][r + 1] = e[1]; hp[2][4 + r] = e2[0]; hp[2][4 + r + 1] = e2[1];
    }
    bf16x8 wc[4][3];
#pragma unroll
    for (int mo = 0; mo < 4; ++mo)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        wc[mo][p] = MRL_FWD_WPF ? wf[mo][p] : w.w1s[(p * 8 + mo * 2 + s) * 64 + lane];
    if (MRL_FWD_WPF && s == 0) load_wf(1);
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      const bf16x8 w0 = wc[mo][0], w1 = wc[mo][1], w2 = wc[mo][2];
      h2[mo] = MFMAB16(w2, hp[0], h2[mo]);  // smallest products first
      h2[mo] = MFMAB16(w0, hp[2], h2[mo]);
      h2[mo] = MFMAB16(w1, hp[1], h2[mo]);
      h2[mo] = MFMAB16(w1, hp[0], h2[mo]);
      h2[mo] = MFMAB16(w0, hp[1], h2[mo]);
      h2[mo] = MFMAB16(w0, hp[0], h2[mo]);
    }
    if (s == 0) {  // the second k-step's activations, under the first one's MFMAs
      tanh4r<BF>(h1[2]);
      tanh4r<BF>(h1[3]);
    }
  }
  if (st != nullptr) st[10] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // tanh + head of output tile mo (head on VALU: 16 units per lane, then the column's 4 rows)
  float acc[A];
#pragma unroll
  for (int o = 0; o < A; ++o) acc[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) {
    tanh4r<BF>(h2[mo]);
#pragma unroll
    for (int o = 0; o < A; ++o) {
      const float4 hv = w.hv[o][mo];
      acc[o] += hv.x * h2[mo][0] + hv.y * h2[mo][1] + hv.z * h2[mo][2] + hv.w * h2[mo][3];
    }
  }
#pragma unroll
  for (int o = 0; o < A; ++o) z[o] = quad_sum(acc[o]) + w.hb[o];
}

// bf16 compute mode on v_mfma_f32_16x16x32_bf16: one k-step covers the inputs, two
// the 64 hidden units (8 MFMAs for layer 1 instead of 64 f32 16x16x4), same rounding
// points as forward16<BF = true> and mlp_rows_bf16.
template <int O, int A, bool BF, class XL>
__device__ inline void forward16(const RWeightsB<O, A>& w, const XL& xl, int lane, float* z, int64_t* st = nullptr) {
  const int g = lane >> 4;
  bf16x8 xb;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) xb[jj] = (__bf16)xl(8 * g + jj);
  f32x4 h1[4], h2[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    h1[m] = as_f32x4(w.b0[m]);
    h2[m] = as_f32x4(w.b1[m]);
  }
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) h1[mo] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.a0[mo], xb, h1[mo], 0, 0, 0);
  if (st != nullptr) st[9] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // B fragment of k-step p: tanh(h1) of tiles 2p (elements 0..3) and 2p+1 (4..7)
  bf16x8 hb[2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      const f32x2 ta = tanh_fast2(f32x2{h1[2 * p][r], h1[2 * p][r + 1]});
      const f32x2 tb = tanh_fast2(f32x2{h1[2 * p + 1][r], h1[2 * p + 1][r + 1]});
      hb[p][r] = (__bf16)ta.x;
      hb[p][r + 1] = (__bf16)ta.y;
      hb[p][4 + r] = (__bf16)tb.x;
      hb[p][4 + r + 1] = (__bf16)tb.y;
    }
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) h2[mo] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.a1[mo][p], hb[p], h2[mo], 0, 0, 0);
  if (st != nullptr) st[10] = (int64_t)__builtin_amdgcn_s_memrealtime();
  float acc[A];
#pragma unroll
  for (int o = 0; o < A; ++o) acc[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 4; ++mo) {
    tanh4r<true>(h2[mo]);
#pragma unroll
    for (int o = 0; o < A; ++o) {
      const float4 hv = w.hv[o][mo];
      acc[o] += hv.x * h2[mo][0] + hv.y * h2[mo][1] + hv.z * h2[mo][2] + hv.w * h2[mo][3];
    }
  }
#pragma unroll
  for (int o = 0; o < A; ++o) z[o] = quad_sum(acc[o]) + w.hb[o];
}

template <int ENV>
__device__ inline void reset_env(const RollArgs& a, int e, double* s) {
  const int E = a.d.n_envs;
  const uint32_t gid = (uint32_t)(a.d.env_offset + e);
  const uint64_t w = (uint64_t)(uint32_t)a.b.env_int[E + e];
  double u[EnvC<ENV>::NU];
#pragma unroll
  for (int c = 0; c < EnvC<ENV>::NU / 2; ++c) philox_uniform2(a.d.seed, 1, gid, w, (uint32_t)c, u[2 * c], u[2 * c + 1]);
  EnvC<ENV>::reset(u, s);
  a.b.env_int[E + e] = (int32_t)(w + 1);
  a.b.env_int[e] = 0;
}

// sum over the 16 lanes of an aligned 16-lane row by DPP (no LDS round trips): lane
// pairs i^1, i^2 (quad_perm), then i <-> 7-i (row_half_mirror), i <-> 15-i (row_mirror);
// every add is commutative in its pair, so all 16 lanes end with the same bits
template <int CTRL>
__device__ inline double dpp_d(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// x / n for an env count n >= 0 (a mean of n values): when every active lane's n is a power
// of two -- a full 64-env block, E = 4096 -- the multiply by the exact 2^-k instead, which is
// the same correctly rounded value as the division (x 2^-k and x / 2^k round the same real
// number once), without the division's dependent v_div_scale / v_rcp / fma chain on the
// step's critical path; the branch is wave-uniform (a ballot)
__device__ inline double div_count(double x, double n) {
  int e;
  const double m = frexp(n, &e);
  if (__builtin_amdgcn_ballot_w64(m != 0.5) == 0) return x * ldexp(1.0, 1 - e);
  return x / n;
}

__device__ inline double sum16(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  return v;
}

// per-block two-pass (mean, M2) partial of vals[ENVS_PER_BLOCK][D] (doubles in LDS):
// thread (k = tid/16, j = tid%16) covers envs j, j+16, ...; 16-lane butterflies.
// column k's (mean, M2) over the block's nvalid envs: lane j adds envs j, j + 16, j + 32,
// j + 48 in that order, then the 16-lane butterflies.  The four values are read from LDS
// together and kept for the M2 pass (one LDS round trip instead of eight dependent ones);
// a term past nvalid is skipped, as the loop over i < nvalid did
__device__ inline void block_moments(const double* vals, int nvalid, int D, int k, int j, double& mean, double& m2) {
  constexpr int Q = ENVS_PER_BLOCK / 16;
  const int kk = k < D ? k : D - 1;
  double v[Q];
  bool in[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int i = j + 16 * q;
    in[q] = k < D && i < nvalid;
    v[q] = vals[(i < nvalid ? i : 0) * D + kk];
  }
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (in[q]) s += v[q];
  mean = nvalid > 0 ? div_count(sum16(s), (double)nvalid) : 0.0;
  double m = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (in[q]) {
      const double dv = v[q] - mean;
      m += dv * dv;
    }
  m2 = sum16(m);
}

__device__ inline void publish_partial(const RollArgs& a, const double* vals, int nvalid, int D, bool with_rew,
                                       double* rec_out) {
  const int k = threadIdx.x >> 4, j = threadIdx.x & 15;
  double mean, m2;
  block_moments(vals, nvalid, D, k, j, mean, m2);
  if (k < D && j == 0) {
    double* r = rec_out + (int64_t)blockIdx.x * a.RS;
    r[2 + k] = mean;
    r[2 + D + k] = m2;
    if (k == 0) {
      r[0] = (double)nvalid;
      r[1] = with_rew ? (double)nvalid : 0.0;
    }
  }
}

// combine the per-block records of one column k into a batch (n, mean, M2):
// mean = sum n_b mean_b / n ; M2 = sum (M2_b + n_b (mean_b - mean)^2).
// Called by all 16 lanes of thread group k; every lane returns the same values.
// Lane j holds records j + 16q of a round (RB_MAX per lane, 128 blocks = 8192 envs).
constexpr int RB_MAX = 8;
template <int R>
struct RecRoundT {
  double rn[R], rm[R], rs[R];
  __device__ void load(const double* rec, int nb, int RS, int D, int O, int k, int j, int b0) {
    const bool isr = (k == O);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int b = b0 + j + 16 * q;
      const double* r = rec + (int64_t)(b < nb ? b : 0) * RS;
      rn[q] = b < nb ? r[isr ? 1 : 0] : 0.0;
      rm[q] = b < nb ? r[2 + k] : 0.0;
      rs[q] = b < nb ? r[2 + D + k] : 0.0;
    }
  }
  __device__ void accumulate(double& n, double& sm, double& raw) const {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      n += rn[q];
      sm += rn[q] * rm[q];
      raw += rs[q] + rn[q] * rm[q] * rm[q];
    }
  }
  // one-round batch (nb <= 16 * R): exact two-pass form from registers
  __device__ void batch(double& bn, double& bm, double& bs) const {
    double n = 0.0, sm = 0.0, raw = 0.0;
    accumulate(n, sm, raw);
    n = sum16(n);
    sm = sum16(sm);
    const double mean = n > 0.0 ? div_count(sm, n) : 0.0;
    double m2 = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (rn[q] > 0.0) {
        const double dm = rm[q] - mean;
        m2 += rs[q] + rn[q] * dm * dm;
      }
    bn = n;
    bm = mean;
    bs = sum16(m2);
  }
};

using RecRound = RecRoundT<RB_MAX>;
// persistent rollout: 16 * RB_SMALL blocks (<= 4096 envs) gather in half the registers
constexpr int RB_SMALL = 4;

__device__ inline void batch_of_records(const double* rec, int nb, int RS, int D, int O, int k, int j, double& bn,
                                        double& bm, double& bs) {
  RecRound rr;
  if (nb <= 16 * RB_MAX) {
    rr.load(rec, nb, RS, D, O, k, j, 0);
    rr.batch(bn, bm, bs);
    return;
  }
  // many rounds: sum (M2_b + n_b mean_b^2) - n mean^2
  double n = 0.0, sm = 0.0, raw = 0.0;
  for (int b0 = 0; b0 < nb; b0 += 16 * RB_MAX) {
    rr.load(rec, nb, RS, D, O, k, j, b0);
    rr.accumulate(n, sm, raw);
  }
  n = sum16(n);
  sm = sum16(sm);
  const double mean = n > 0.0 ? div_count(sm, n) : 0.0;
  bn = n;
  bm = mean;
  bs = sum16(raw) - n * mean * mean;
}

// Chan merge of (nb, mb, m2b) into (n, M, S); for nb == 1 this is RunningStat.push
// the filtered observation columns 4i + g of one env row (core.py:191-192: clip((o - mean)
// / (std + 1e-8), -5, 5)), as f32.  Every column's statistics are read from LDS before any
// arithmetic and the stores are left to the caller, so the (O + 3) / 4 divisions are
// independent chains rather than one LDS round trip + division per branchy store block
// (the same operations per value)
template <int ENV>
__device__ inline void filtered_obs(const double* s, int g, bool filter, const double* fmean, const double* fden,
                                    float* vf) {
  constexpr int O = EnvC<ENV>::OBS, NI = (O + 3) / 4;
  double o[O];
  EnvC<ENV>::obs(s, o);
  double v[NI], mu[NI], den[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    v[i] = o[4 * i];
#pragma unroll
    for (int q = 1; q < 4; ++q)
      if (4 * i + q < O && g == q) v[i] = o[4 * i + q < O ? 4 * i + q : O - 1];
  }
  if (filter) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int kc = 4 * i + g, kk = kc < O ? kc : O - 1;
      mu[i] = fmean[kk];
      den[i] = fden[kk];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      double x = v[i] - mu[i];
      x = x / den[i];
      v[i] = x < -5.0 ? -5.0 : (x > 5.0 ? 5.0 : x);
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) vf[i] = (float)v[i];
}

__device__ inline void chan_merge(double& n, double& M, double& S, double nb, double mb, double m2b) {
  if (nb <= 0.0) return;
  const double na = n;
  const double nn = na + nb;
  const double delta = mb - M;
  const double newM = M + (delta * nb) / nn;
  S = S + m2b + delta * (mb - newM) * nb;
  M = newM;
  n = nn;
}

// Sampling noise of env e at step t is Philox (gid, iteration*T + t) on domain 0:
// Categorical u = first uniform of call 0, Gauss z[2c], z[2c+1] = Box-Muller of call
// c.  A whole iteration's rows are drawn up front by noise_fill_kernel (one thread per
// (row, pair): the transcendental work leaves the step kernels' latency chain), or
// injected by the caller; the step kernels only load zn rows.
template <int ENV>
__device__ inline void load_noise(const RollArgs& a, int64_t row, double* zn) {
  using EC = EnvC<ENV>;
  const double* nz = reinterpret_cast<const double*>(a.b.noise);
  if constexpr (EC::DISCRETE) zn[0] = nz[row];
  else
#pragma unroll
    for (int q = 0; q < EC::ACT; ++q) zn[q] = nz[row * EC::ACT + q];
}

template <int ENV>
__global__ void noise_fill_kernel(RollArgs a, double* __restrict__ out) {
  using EC = EnvC<ENV>;
  constexpr int A = EC::ACT, P = EC::DISCRETE ? 1 : (A + 1) / 2;
  // grid (ceil(E * P / 256), min(T, 65535)): steps t = blockIdx.y + k * gridDim.y, no runtime
  // 64-bit division
  const int E = a.d.n_envs;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E * P) return;
  const int c = i % P, e = i / P;
  for (int t = blockIdx.y; t < a.d.horizon; t += gridDim.y) {
    const int64_t row = (int64_t)t * E + e;
    const uint32_t gid = (uint32_t)(a.d.env_offset + e);
    const uint64_t w = (uint64_t)(*a.b.iteration) * (uint64_t)a.d.horizon + (uint64_t)t;
    double u0, u1;
    philox_uniform2(a.d.seed, 0, gid, w, (uint32_t)c, u0, u1);
    if constexpr (EC::DISCRETE) {
      out[row] = u0;
    } else {
      const double rad = sqrt(-2.0 * log(1.0 - u0));
      double sn, cn;
      sincos(2.0 * 3.141592653589793 * u1, &sn, &cn);
      out[row * A + 2 * c] = rad * cn;
      if (2 * c + 1 < A) out[row * A + 2 * c + 1] = rad * sn;
    }
  }
}

// sample the action from the head rows z (core.py:261-267; distributions.py:3-13 /
// core.py:432-435), write act/prob rows, step the env (fp64)
// QUAD: the four 16-lane rows of the wave hold this env (fused step kernel); every
// lane steps it (row h = lane >> 4 of the angle functions), lanes with `store` write
// SD: `logstd` holds the standard deviations exp(logstd) already (the persistent kernel
// forms them once per launch: the same expf, not one per step)
template <int ENV, bool QUAD = false, bool SD = false>
__device__ inline void sample_and_step(const RollArgs& a, int64_t row, const float* z, const float* logstd,
                                       const double* zn, double* s, double& rew, bool& done, bool store = true,
                                       int h = 0, const double* capc = nullptr) {
  using EC = EnvC<ENV>;
  constexpr int A = EC::ACT;
  if constexpr (EC::DISCRETE) {
    float m = z[0];
#pragma unroll
    for (int q = 1; q < A; ++q) m = fmaxf(m, z[q]);
    float p[A], se = 0.f;
#pragma unroll
    for (int q = 0; q < A; ++q) {
      p[q] = expf(z[q] - m);
      se += p[q];
    }
#pragma unroll
    for (int q = 0; q < A; ++q) p[q] = p[q] / se;
    const double u = zn[0];
    int act = 0;
    float cs = 0.f;
    bool found = false;
#pragma unroll
    for (int q = 0; q < A; ++q) {
      cs += p[q];
      if (!found && (double)cs > u) {
        act = q;
        found = true;
      }
    }
    if (store) {
      reinterpret_cast<int32_t*>(a.b.act)[row] = act;
#pragma unroll
      for (int q = 0; q < A; ++q) a.b.prob[row * A + q] = p[q];
    }
    EC::step_disc(s, act, rew, done);
  } else {
    float av[A];
#pragma unroll
    for (int q = 0; q < A; ++q) {
      const float sd = SD ? logstd[q] : expf(logstd[q]);
      av[q] = __fadd_rn(__fmul_rn((float)zn[q], sd), z[q]);
      if (store) {
        reinterpret_cast<float*>(a.b.act)[row * A + q] = av[q];
        a.b.prob[row * 2 * A + q] = z[q];
        a.b.prob[row * 2 * A + A + q] = sd;
      }
    }
    if constexpr (QUAD) EC::step_cont_quad(s, av, rew, done, h, capc);
    else EC::step_cont(s, av, rew, done);
  }
}

// episode bookkeeping: gym TimeLimit => done (terminated, bootstrap 0); the rollout
// loop limit / horizon cut => not terminated (core.py:190-207, 73); auto-reset; store
template <int ENV>
__device__ inline void finish_env_step(const RollArgs& a, int e, int64_t row, int t, double* s, double rew, bool done) {
  using EC = EnvC<ENV>;
  const int E = a.d.n_envs;
  const int ept = a.b.env_int[e];
  a.b.ep_t[row] = ept;
  const bool term = done || (ept + 1 >= EC::MAX_STEPS);
  const bool last = term || (ept + 1 >= a.d.timestep_limit) || (t == a.d.horizon - 1);
  a.b.rew[row] = (float)rew;
  a.b.flags[row] = (uint8_t)((last ? 1 : 0) | (term ? 2 : 0));
  if (last && t < a.d.horizon - 1) reset_env<ENV>(a, e, s);
  else a.b.env_int[e] = ept + 1;
#pragma unroll
  for (int i = 0; i < EC::NS; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
}

template <int ENV>
__global__ __launch_bounds__(RB) void rollout_reset_kernel(RollArgs a) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS, D = O + 1;
  __shared__ double vals[ENVS_PER_BLOCK * MAXD];
  const int E = a.d.n_envs;
  const int le = threadIdx.x;
  const int e = blockIdx.x * ENVS_PER_BLOCK + le;
  if (le < ENVS_PER_BLOCK && e < E) {
    double s[EC::NS], o[O];
    reset_env<ENV>(a, e, s);
#pragma unroll
    for (int i = 0; i < EC::NS; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
    EC::obs(s, o);
#pragma unroll
    for (int k = 0; k < O; ++k) vals[le * D + k] = o[k];
    vals[le * D + O] = 0.0;
  }
  __syncthreads();
  const int nvalid = min(ENVS_PER_BLOCK, E - (int)blockIdx.x * ENVS_PER_BLOCK);
  publish_partial(a, vals, nvalid, D, false, a.b.records);
}

// rollout image: rimage_value (mlp_layout.h) of every element
// part p (0, 1, 2) of an f32 value's exact three-way bf16 split (mlp_split.hip)
__device__ inline float rb_part(float v, int p) {
  const __bf16 a = (__bf16)v;
  if (p == 0) return (float)a;
  const float r = v - (float)a;
  const __bf16 c = (__bf16)r;
  if (p == 1) return (float)c;
  return r - (float)c;
}

__global__ void rollout_pack_kernel(RDims r, MlpDims d, const float* __restrict__ th, float* __restrict__ out,
                                    int bf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < r.f32_size) {
    const float v = rimage_value(r, d, th, i);
    out[i] = (bf && i < r.b0) ? bf16r(v) : v;  // bf16 mode: the MFMA weights W0, W1
  } else if (i >= r.bs1 && i < r.size) {
    // split W1 fragments (fp32 mode): part p of the ba1 fragment elements, two per word
    const int rel = i - r.bs1, part = rel / (4 * 2 * 64 * 4), rr = rel % (4 * 2 * 64 * 4);
    const int frag = rr >> 2, q = rr & 3;
    const __bf16 lo = (__bf16)rb_part(rimage_bf16_elem(d, th, true, frag, 2 * q), part);
    const __bf16 hi = (__bf16)rb_part(rimage_bf16_elem(d, th, true, frag, 2 * q + 1), part);
    out[i] = __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, lo) |
                             ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16));
  } else if (i < r.size) {
    // bf16 fragments: two bf16 per word
    const bool l1 = i >= r.ba1;
    const int rel = i - (l1 ? r.ba1 : r.ba0), frag = rel >> 2, q = rel & 3;
    const __bf16 lo = (__bf16)rimage_bf16_elem(d, th, l1, frag, 2 * q);
    const __bf16 hi = (__bf16)rimage_bf16_elem(d, th, l1, frag, 2 * q + 1);
    out[i] = __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, lo) |
                             ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16));
  }
}

// One launch = step t of E envs: 4 waves x 16 envs per block, the four 16-lane rows of
// a wave share the wave's 16 envs (split angle functions / noise / obs columns, the
// MFMA tiles of forward16).
template <int ENV, bool BF>
__global__ __launch_bounds__(RB) void rollout_step_kernel(RollArgs a, const float* __restrict__ logstd,
                                                          const float* __restrict__ rimg, int t) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS, D = O + 1, NS = EC::NS, A = EC::ACT;
  __shared__ double vals[ENVS_PER_BLOCK * MAXD];
  __shared__ double fmean[MAXD], fden[MAXD];
  __shared__ float xt[4][16][MAX_IN + 1];  // +1: conflict-free column reads
  // diagnostic phase stamps (100 MHz realtime) of block 0 / thread 0 -- never set in production
#define STAMP(k)                                                                    \
  do {                                                                              \
    if (a.b.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0)               \
      a.b.stamps[(int64_t)t * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
  STAMP(0);
  if (a.b.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0)  // shader clock, for the in-kernel GHz
    a.b.stamps[(int64_t)t * 16 + 14] = (int64_t)__builtin_amdgcn_s_memtime();
  const int E = a.d.n_envs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int le = wave * 16 + j;
  const int e = blockIdx.x * ENVS_PER_BLOCK + le;
  const bool valid = e < E;
  const int64_t row = (int64_t)t * E + e;

  // 0. every global load of the step up front, in the order they are consumed (the
  //    vector-memory counter retires in order): filter records, env state, noise
  //    rows, policy weights
  const double* fs_in = a.b.filter_state + (t & 1) * a.FS;
  double* fs_out = a.b.filter_state + ((t + 1) & 1) * a.FS;
  const double* rec_in = a.b.records + (int64_t)(t & 1) * a.nb * a.RS;
  double* rec_out = a.b.records + (int64_t)((t + 1) & 1) * a.nb * a.RS;
  const int k = threadIdx.x >> 4, jj = threadIdx.x & 15;
  const bool kcol = k < D, isr = (k == O), one_round = a.nb <= 16 * RB_MAX;
  RecRound rr;
  double fn = 0.0, fM = 0.0, fS = 0.0;
  if (kcol) {
    if (one_round) rr.load(rec_in, a.nb, a.RS, D, O, k, jj, 0);
    fn = fs_in[isr ? 1 : 0];
    fM = fs_in[2 + k];
    fS = fs_in[2 + D + k];
  }
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = valid ? a.b.env_state[(int64_t)i * E + e] : 0.0;
  double zn[A + 1] = {};
  if (valid) load_noise<ENV>(a, row, zn);
  RollWeights<O, A, BF> wt;
  wt.load(rimg, lane);
  __shared__ bf16x8 w1s_l[BF ? 1 : 3 * 8 * 64];  // fp32 mode: the split W1 fragments (24 KB)
  if constexpr (!BF) {
    constexpr RDims R = rollout_dims(O);
    for (int i = threadIdx.x; i < 3 * 8 * 64; i += RB) w1s_l[i] = reinterpret_cast<const bf16x8*>(rimg + R.bs1)[i];
    wt.w1s = w1s_l;
  }
  float lsd[A];
#pragma unroll
  for (int q = 0; q < A; ++q) lsd[q] = EC::DISCRETE ? 0.f : logstd[q];
  STAMP(1);

  // 2. running-stat merge (filters.py:30-31 push, per step over all envs): the block
  //    partials -> one batch -> one Chan merge; every block derives the same state
  if (kcol) {
    double bn, bm, bs;
    if (one_round) rr.batch(bn, bm, bs);
    else batch_of_records(rec_in, a.nb, a.RS, D, O, k, jj, bn, bm, bs);
    chan_merge(fn, fM, fS, bn, bm, bs);
    if (jj == 0 && blockIdx.x == 0) {
      if (k == 0) fs_out[0] = fn;
      if (isr) fs_out[1] = fn;
      fs_out[2 + k] = fM;
      fs_out[2 + D + k] = fS;
    }
    if (!isr && jj == 0) {
      const double var = fn > 1.0 ? fS / (fn - 1.0) : fM * fM;  // running_stat.py:27
      fmean[k] = fM;
      fden[k] = sqrt(var) + 1e-8;
    }
  }
  __syncthreads();
  STAMP(2);

  // 3. filtered observation (core.py:191-192); row g takes columns 4i + g
  {
    float vf[(O + 3) / 4];
    filtered_obs<ENV>(s, g, a.d.filter != 0, fmean, fden, vf);
#pragma unroll
    for (int i = 0; i < (O + 3) / 4; ++i) {
      const int kc = 4 * i + g;
      if (kc < O) {
        if (valid) a.b.obs[row * O + kc] = vf[i];
        xt[wave][j][kc] = vf[i];
      }
    }
  }
  WAVE_LDS_ORDER();
  STAMP(3);

  // 4. policy forward (MFMA, 16 envs per wave)
  struct XL {
    const float* p;
    bool valid;
    __device__ inline float operator()(int c) const { return (valid && c < O) ? p[c] : 0.f; }
  } xl{&xt[wave][j][0], valid};
  float z[A];
  forward16<O, A, BF>(wt, xl, lane, z,
                  (a.b.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0) ? a.b.stamps + t * 16 : nullptr);
  STAMP(4);

  // 5. sample + env step: every row steps the env (split angle functions), row 0 stores
  double rew = 0.0;
  bool done = false;
  sample_and_step<ENV, true>(a, row, z, lsd, zn, s, rew, done, valid && g == 0, g);
  STAMP(5);
  if (valid && g == 0) {
    finish_env_step<ENV>(a, e, row, t, s, rew, done);
    // 6. raw next observation + reward into the block partial
    double o[O];
    EC::obs(s, o);
#pragma unroll
    for (int c = 0; c < O; ++c) vals[le * D + c] = o[c];
    vals[le * D + O] = rew;
  }
  __syncthreads();
  STAMP(6);
  const int nvalid = min(ENVS_PER_BLOCK, E - (int)blockIdx.x * ENVS_PER_BLOCK);
  publish_partial(a, vals, nvalid, D, true, rec_out);
  STAMP(7);
  if (a.b.stamps != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    a.b.stamps[(int64_t)t * 16 + 15] = (int64_t)__builtin_amdgcn_s_memtime();
#undef STAMP
}

// ------------------------------------------------------------------ persistent rollout
// The whole horizon in ONE launch (mrl_rollout_run): the nb blocks of the step kernel
// stay resident (one block per CU of the launch stream's CU set) and loop over t.  Weights, env state, episode
// counters and the running stat live in registers for all T steps; the only cross-block
// dependency of a step -- the Welford partials of the E raw observations (and rewards)
// that every block merges into its copy of the running stat -- is handed off in memory
// as data-tagged granules: each (block, column) partial is ONE 16-B granule {fp64 mean,
// fp64 M2} written by a single write-through (sc1) store, the step tag riding in M2's
// sign bit (M2 >= 0); a consumer polls the granules themselves with sc1 loads until
// every tag carries the step it waits for, so one memory round trip both signals and
// delivers (MI355X_MICROARCH.md, hand-offs: untorn 16-B sc1 granules).  Counts are not
// sent: every block knows each block's number of envs.  Two parities as between step
// launches: block b can only overwrite the parity-p granule of gather step s at step
// s+2 after every block's step-s+1 granules arrived, i.e. after every block has read
// step s; so a slot only ever holds step s or s-2 (or the launch's memset zeros), and
// one tag bit that alternates between consecutive writes of a slot -- tag(s) =
// ((s >> 1) & 1) ^ 1, never the memset's 0 for s = 0, 1 -- tells them apart.
// Bit-identical to the step kernels.
constexpr int SYNC_ABORT = 32;             // u32 word: a block gave up waiting (own 128-B line)
constexpr int64_t SYNC_HEAD_BYTES = 256;   // then the granules: [2 parities][D][nb] x 16 B
constexpr uint32_t SPIN_LIMIT = 1u << 22;  // polls (~seconds): a non-resident grid exits

typedef uint32_t gran_t __attribute__((ext_vector_type(4)));  // one 16-B granule

__device__ inline uint32_t step_tag(int s) { return (((uint32_t)s >> 1) & 1u) ^ 1u; }

struct Granules {
  __amdgpu_buffer_rsrc_t rsrc;
  int nb, D;
  __device__ Granules(uint32_t* sync, int nb_, int D_) : nb(nb_), D(D_) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(sync) + SYNC_HEAD_BYTES, 0,
                                             2 * D_ * nb_ * 16, 0x00020000);
  }
  __device__ uint32_t off(int parity, int k, int b) const { return (uint32_t)(((parity * D + k) * nb + b) * 16); }
  __device__ void put(int step, int k, int b, double mean, double m2) const {
    const uint64_t mb = (uint64_t)__double_as_longlong(mean);
    const uint64_t sb = ((uint64_t)__double_as_longlong(m2) & ~(1ull << 63)) | ((uint64_t)step_tag(step) << 63);
    gran_t g = {(uint32_t)mb, (uint32_t)(mb >> 32), (uint32_t)sb, (uint32_t)(sb >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(g, rsrc, off(step & 1, k, b), 0, 16);  // aux 16 = sc1
  }
  __device__ gran_t get(int step, int k, int b) const {
    return __builtin_amdgcn_raw_buffer_load_b128(rsrc, off(step & 1, k, b), 0, 16);
  }
};
__device__ inline double g_mean(gran_t g) { return __longlong_as_double((long long)(((uint64_t)g.y << 32) | g.x)); }
__device__ inline double g_m2(gran_t g) {
  return __longlong_as_double((long long)((((uint64_t)(g.w & 0x7fffffffu)) << 32) | g.z));
}
__device__ inline bool g_tag_is(gran_t g, int step) { return (g.w >> 31) == step_tag(step); }

// the block's (mean, M2) partial of vals[nvalid][D] (publish_partial's arithmetic) as
// the granules of gather step `step`; lane 0 of column group k writes column k's
__device__ inline void publish_granules(const Granules& gr, const double* vals, int nvalid, int step) {
  const int k = threadIdx.x >> 4, j = threadIdx.x & 15;
  double mean, m2;
  block_moments(vals, nvalid, gr.D, k, j, mean, m2);
  if (k < gr.D && j == 0) gr.put(step, k, blockIdx.x, mean, m2);
}

// column k's records of blocks b0 + jj + 16q as RecRound registers, polled until every
// granule carries gather step `step`'s tag; n_b is known (envs of block b; 0 for the
// reward column of the reset partial).  false: the grid gave up (some block never
// published).
template <int R, class Under>
__device__ inline bool gather_granules(const Granules& gr, RecRoundT<R>& rr, int step, int k, int jj, int b0, int E,
                                       bool rew_counted, uint32_t* sync, Under&& under) {
  const bool isr = (k == gr.D - 1);
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int b = b0 + jj + 16 * q;
    rr.rn[q] = (b < gr.nb && (!isr || rew_counted)) ? (double)min(ENVS_PER_BLOCK, E - b * ENVS_PER_BLOCK) : 0.0;
  }
  uint32_t it = 0;
  while (true) {
    gran_t gq[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int b = b0 + jj + 16 * q;
      gq[q] = gr.get(step, k, b < gr.nb ? b : 0);
    }
    if (it == 0) under();  // independent work while the first poll's loads are in flight
    bool ready = true;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const bool in = b0 + jj + 16 * q < gr.nb;
      ready = ready && (!in || g_tag_is(gq[q], step));
      rr.rm[q] = in ? g_mean(gq[q]) : 0.0;
      rr.rs[q] = in ? g_m2(gq[q]) : 0.0;
    }
    if (ready) return true;
    __builtin_amdgcn_s_sleep(1);
    if ((++it & 255) == 0 &&
        (it > SPIN_LIMIT || __hip_atomic_load(sync + SYNC_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      __hip_atomic_store(sync + SYNC_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// initial state of env e's episode number epc (reset_env's Philox draw, domain 1)
template <int ENV>
__device__ inline void episode_start_state(const RollArgs& a, int e, uint32_t epc, double* s) {
  const uint32_t gid = (uint32_t)(a.d.env_offset + e);
  double u[EnvC<ENV>::NU];
#pragma unroll
  for (int c = 0; c < EnvC<ENV>::NU / 2; ++c)
    philox_uniform2(a.d.seed, 1, gid, (uint64_t)epc, (uint32_t)c, u[2 * c], u[2 * c + 1]);
  EnvC<ENV>::reset(u, s);
}

// ST: the diagnostic build with phase stamps (launched only when bufs.stamps is set);
// production launches carry no stamp code, whose uniform pointers / offsets cost SGPRs
// that the compiler then spilled to VGPR lanes (a v_readlane per reload, every step).
template <int ENV, bool BF, bool ST>
__global__ __launch_bounds__(RB) void rollout_persistent_kernel(RollArgs a, const float* __restrict__ logstd,
                                                                const float* __restrict__ rimg,
                                                                uint32_t* __restrict__ sync) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS, D = O + 1, NS = EC::NS, A = EC::ACT;
  __shared__ double vals[ENVS_PER_BLOCK * MAXD];
  __shared__ double fmean[MAXD], fden[MAXD];
  __shared__ float xt[4][16][MAX_IN + 1];  // +1: conflict-free column reads
  __shared__ int s_fail;
  // HP_CAP: the capsule constants, one LDS read per constant per substep instead of a
  // select chain on the lane's row (rollout 14.30 -> 14.05 ms, profiles/r06d_ab.txt)
  __shared__ double hp_cap[24];
  const int E = a.d.n_envs, T = a.d.horizon, nb = a.nb;
  // diagnostic phase stamps (100 MHz realtime) of block 0 -- never set in production
#define PSTAMP(tt, k)                                                                  \
  do {                                                                                 \
    if (ST && threadIdx.x == 0 && blockIdx.x == 0)                                     \
      a.b.stamps[(int64_t)(tt) * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int le = wave * 16 + j;
  const int e = blockIdx.x * ENVS_PER_BLOCK + le;
  const bool valid = e < E;
  const int ec = valid ? e : E - 1;  // invalid lanes shadow a valid env, store nothing
  const int k = threadIdx.x >> 4, jj = threadIdx.x & 15;
  const bool kcol = k < D, isr = (k == O);
  const int nvalid = min(ENVS_PER_BLOCK, E - (int)blockIdx.x * ENVS_PER_BLOCK);
  const Granules gr(sync, nb, D);
  if (threadIdx.x == 0) s_fail = 0;
  if (threadIdx.x < 24) hp_cap[threadIdx.x] = HP_CAP[threadIdx.x];

  RollWeights<O, A, BF> wt;
  wt.load(rimg, lane);
  __shared__ bf16x8 w1s_l[BF ? 1 : 3 * 8 * 64];  // fp32 mode: the split W1 fragments (24 KB)
  if constexpr (!BF) {
    constexpr RDims R = rollout_dims(O);
    for (int i = threadIdx.x; i < 3 * 8 * 64; i += RB) w1s_l[i] = reinterpret_cast<const bf16x8*>(rimg + R.bs1)[i];
    wt.w1s = w1s_l;
  }
  float lsd[A], sdv[A];
#pragma unroll
  for (int q = 0; q < A; ++q) {
    lsd[q] = EC::DISCRETE ? 0.f : logstd[q];
    sdv[q] = expf(lsd[q]);
  }
  // the running stat at the start of the iteration (every block keeps the same copy)
  double fn = 0.0, fM = 0.0, fS = 0.0;
  if (kcol) {
    fn = a.b.filter_state[isr ? 1 : 0];
    fM = a.b.filter_state[2 + k];
    fS = a.b.filter_state[2 + D + k];
  }
  // reset every env (core.py:186); all four rows of a wave hold the same env.  sn is
  // the start state of the env's NEXT episode, drawn ahead so an auto-reset is a copy:
  // its Philox draw runs behind the step's publish, under the hand-off latency.
  double s[NS], sn[NS];
  uint32_t epc = (uint32_t)a.b.env_int[E + ec];
  int ept = 0;
  episode_start_state<ENV>(a, ec, epc, s);
  epc += 1u;
  episode_start_state<ENV>(a, ec, epc, sn);
  bool refill = false;
  if (valid && g == 0) {
    double o[O];
    EC::obs(s, o);
#pragma unroll
    for (int c = 0; c < O; ++c) vals[le * D + c] = o[c];
    vals[le * D + O] = 0.0;
  }
  __syncthreads();
  publish_granules(gr, vals, nvalid, 0);  // gather step 0's partials
  double capr[6];  // row g's capsule constants (MRL_HP_CAP_LDS 2)
#pragma unroll
  for (int f = 0; f < 6; ++f) capr[f] = hp_cap[4 * f + g];

  for (int t = 0; t < T; ++t) {
    const int64_t row = (int64_t)t * E + e;
    PSTAMP(t, 0);
    if (ST && threadIdx.x == 0 && blockIdx.x == 0)  // shader clock beside the 100 MHz one (in-kernel GHz)
      a.b.stamps[(int64_t)t * 16 + 9] = (int64_t)__builtin_amdgcn_s_memtime();
    double zn[A + 1] = {};
    load_noise<ENV>(a, (int64_t)t * E + ec, zn);  // independent of the hand-off: issued first
    // the next episode's start state of envs that auto-reset at step t-1: off the step's
    // critical path, under the first poll of the hand-off (or beside it, non-polling waves)
    auto refill_next = [&]() {
      if (refill) {
        episode_start_state<ENV>(a, ec, epc, sn);
        refill = false;
      }
    };
    // running-stat merge of step t's batch (filters.py:30-31), identical in every block
    if (!kcol) refill_next();  // kcol is wave-uniform: waves that do not poll
    if (kcol) {
      double bn, bm, bs;
      RecRound rr;
      bool ok = true;
      if (nb <= 16 * RB_SMALL) {
        RecRoundT<RB_SMALL> r4;
        ok = gather_granules(gr, r4, t, k, jj, 0, E, t > 0, sync, refill_next);
        PSTAMP(t, 7);
        r4.batch(bn, bm, bs);
      } else if (nb <= 16 * RB_MAX) {
        ok = gather_granules(gr, rr, t, k, jj, 0, E, t > 0, sync, refill_next);
        PSTAMP(t, 7);
        rr.batch(bn, bm, bs);
      } else {
        double n = 0.0, sm = 0.0, raw = 0.0;
        for (int b0 = 0; b0 < nb && ok; b0 += 16 * RB_MAX) {
          ok = gather_granules(gr, rr, t, k, jj, b0, E, t > 0, sync, refill_next);
          rr.accumulate(n, sm, raw);
        }
        n = sum16(n);
        sm = sum16(sm);
        bm = n > 0.0 ? div_count(sm, n) : 0.0;
        bn = n;
        bs = sum16(raw) - n * bm * bm;
      }
      if (!ok) s_fail = 1;
      chan_merge(fn, fM, fS, bn, bm, bs);
      if (!isr && jj == 0) {
        const double var = fn > 1.0 ? fS / (fn - 1.0) : fM * fM;  // running_stat.py:27
        fmean[k] = fM;
        fden[k] = sqrt(var) + 1e-8;
      }
    }
    PSTAMP(t, 8);
    __syncthreads();
    if (s_fail) break;  // uniform: a block that gave up leaves the loop whole
    PSTAMP(t, 1);
    // filtered observation (core.py:191-192); row g takes columns 4i + g
    {
      float vf[(O + 3) / 4];
      filtered_obs<ENV>(s, g, a.d.filter != 0, fmean, fden, vf);
#pragma unroll
      for (int i = 0; i < (O + 3) / 4; ++i) {
        const int kc = 4 * i + g;
        if (kc < O) {
          if (valid) a.b.obs[row * O + kc] = vf[i];
          xt[wave][j][kc] = vf[i];
        }
      }
    }
    WAVE_LDS_ORDER();
    PSTAMP(t, 2);
    struct XL {
      const float* p;
      bool valid;
      __device__ inline float operator()(int c) const { return (valid && c < O) ? p[c] : 0.f; }
    } xl{&xt[wave][j][0], valid};
    float z[A];
    forward16<O, A, BF>(wt, xl, lane, z);
    PSTAMP(t, 3);
    // sample + env step on every row (split angle functions); row 0 stores
    double rew = 0.0;
    bool done = false;
    sample_and_step<ENV, true, true>(a, row, z, sdv, zn, s, rew, done, valid && g == 0, g,
                                     MRL_HP_CAP_LDS == 2 ? capr : hp_cap);
    PSTAMP(t, 4);
    // episode bookkeeping on every row, so the rows keep identical env state
    // (finish_env_step: gym TimeLimit => terminated; limit / horizon cut => not)
    {
      const bool term = done || (ept + 1 >= EC::MAX_STEPS);
      const bool last = term || (ept + 1 >= a.d.timestep_limit) || (t == T - 1);
      if (valid && g == 0) {
        a.b.ep_t[row] = ept;
        a.b.rew[row] = (float)rew;
        a.b.flags[row] = (uint8_t)((last ? 1 : 0) | (term ? 2 : 0));
      }
      if (last && t < T - 1) {
#pragma unroll
        for (int i = 0; i < NS; ++i) s[i] = sn[i];
        epc += 1u;
        ept = 0;
        refill = true;
      } else {
        ept += 1;
      }
    }
    if (valid && g == 0) {
      double o[O];
      EC::obs(s, o);
#pragma unroll
      for (int c = 0; c < O; ++c) vals[le * D + c] = o[c];
      vals[le * D + O] = rew;
    }
    __syncthreads();
    PSTAMP(t, 5);
    if (t + 1 < T) publish_granules(gr, vals, nvalid, t + 1);
    else publish_partial(a, vals, nvalid, D, true, a.b.records + (int64_t)(T & 1) * nb * a.RS);  // for finish
    PSTAMP(t, 6);
  }
#undef PSTAMP
  // state for the next iteration and the finish kernel: env state / counters, and the
  // running stat where the step kernels leave it (parity T)
  if (valid && g == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
    a.b.env_int[e] = ept;
    a.b.env_int[E + e] = (int32_t)epc;
  }
  if (blockIdx.x == 0 && kcol && jj == 0) {
    double* fs_out = a.b.filter_state + (T & 1) * a.FS;
    if (k == 0) fs_out[0] = fn;
    if (isr) fs_out[1] = fn;
    fs_out[2 + k] = fM;
    fs_out[2 + D + k] = fS;
  }
}

// ------------------------------------------------------------------ layered-policy rollout
// For policies the fused step kernel does not cover (wide nets, Humanoid's 376-d obs),
// step t is three launches: lrollout_obs (filter merge + normalised obs rows) ->
// the policy's GEMM forward over the E rows (LayeredMlpNet) -> lrollout_act (sample,
// env step, raw next obs + reward as SoA rows [O+1][E] fp64, block partials).
constexpr int MAXD_L = 384;  // obs dims + 1 on the layered path

// Layered-path kernels are parallel over (env block, 32-column chunk): the 376-d obs
// makes every per-column loop long, so no block walks all columns.
constexpr int LCOLS = 32;

// per-(env block, column chunk) two-pass partial of the SoA rows raw[k][e0 .. e0+nvalid):
// column k = 32*blockIdx.y + (tid & 31); 8 thread groups stride the envs.
__global__ __launch_bounds__(RB) void lrollout_partials_kernel(RollArgs a, int D, int rec_parity, int with_rew) {
  __shared__ double red[8][LCOLS];
  const int E = a.d.n_envs;
  const int e0 = blockIdx.x * ENVS_PER_BLOCK;
  const int nvalid = min(ENVS_PER_BLOCK, E - e0);
  const int c = threadIdx.x & (LCOLS - 1), g = threadIdx.x >> 5;
  const int k = blockIdx.y * LCOLS + c;
  double* r = a.b.records + (int64_t)rec_parity * a.nb * a.RS + (int64_t)blockIdx.x * a.RS;
  const double* col = a.b.raw_obs + (int64_t)(k < D ? k : 0) * E + e0;
  // this thread's values (rows g, g + 8, ...) loaded once, all issued together, for both
  // passes; the sums stay in row order
  constexpr int PR = ENVS_PER_BLOCK / 8;
  double cv[PR];
#pragma unroll
  for (int q = 0; q < PR; ++q) cv[q] = col[min(g + 8 * q, max(nvalid - 1, 0))];  // clamped: in the column
  double sm = 0.0;
  if (k < D)
#pragma unroll
    for (int q = 0; q < PR; ++q)
      if (g + 8 * q < nvalid) sm += cv[q];
  red[g][c] = sm;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) tot += red[q][c];
  const double mean = nvalid > 0 ? div_count(tot, (double)nvalid) : 0.0;
  __syncthreads();
  double m2 = 0.0;
  if (k < D)
#pragma unroll
    for (int q = 0; q < PR; ++q)
      if (g + 8 * q < nvalid) {
        const double dv = cv[q] - mean;
        m2 += dv * dv;
      }
  red[g][c] = m2;
  __syncthreads();
  if (g == 0 && k < D) {
    double t2 = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) t2 += red[q][c];
    r[2 + k] = mean;
    r[2 + D + k] = t2;
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    r[0] = (double)nvalid;
    r[1] = with_rew ? (double)nvalid : 0.0;
  }
}

template <int ENV>
__global__ __launch_bounds__(RB) void lrollout_reset_kernel(RollArgs a) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS;
  const int E = a.d.n_envs;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) {
    double s[EC::NS];
    reset_env<ENV>(a, e, s);
#pragma unroll
    for (int i = 0; i < EC::NS; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
    double* raw = a.b.raw_obs;
    EC::obs_out(s, [&](int k, double v) { raw[(int64_t)k * E + e] = v; });
    raw[(int64_t)O * E + e] = 0.0;
  }
}

// merge of the batch records (block order, two passes: n, mean = sum n_b m_b / n,
// M2 = sum M2_b + n_b (m_b - mean)^2 -- oracle/rollout_np.py _batch) into the running
// stat, then the normalised obs rows of step t for this (env block, column chunk)
template <int ENV>
__global__ __launch_bounds__(RB) void lrollout_obs_kernel(RollArgs a, int t) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS, D = O + 1;
  __shared__ double fmean[LCOLS], fden[LCOLS];
  constexpr int G = RB / ENVS_PER_BLOCK, CPT = LCOLS / G;  // thread groups over columns, columns per thread
  static_assert(RB % ENVS_PER_BLOCK == 0 && LCOLS % G == 0, "tile mapping");
  __shared__ float tile[LCOLS * (ENVS_PER_BLOCK + 1)];
  const int E = a.d.n_envs;
  const double* fs_in = a.b.filter_state + (t & 1) * a.FS;
  double* fs_out = a.b.filter_state + ((t + 1) & 1) * a.FS;
  const double* rec = a.b.records + (int64_t)(t & 1) * a.nb * a.RS;
  const int kbase = blockIdx.y * LCOLS;
  // this block's raw observation values, loaded first: their latency runs under the
  // record loads and the merge below (they do not depend on it)
  const int e0 = blockIdx.x * ENVS_PER_BLOCK;
  const int nvalid = min(ENVS_PER_BLOCK, E - e0);
  const int el = threadIdx.x % ENVS_PER_BLOCK, kb = threadIdx.x / ENVS_PER_BLOCK;
  double v[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const int k = kbase + kb + G * q;
    v[q] = (k < O && el < nvalid) ? a.b.raw_obs[(int64_t)k * E + e0 + el] : 0.0;
  }
  if (threadIdx.x < LCOLS && kbase + (int)threadIdx.x < D) {
    const int k = kbase + threadIdx.x;
    const bool isr = (k == O);
    // the block records in chunks of LREC: every load of a chunk issued before the
    // chunk's sums (the sums themselves stay sequential in block order, as the oracle's);
    // one dependent global load per block per pass had made this launch ~14 us of waiting
    constexpr int LREC = 16;
    double bn = 0.0, sm = 0.0, bm = 0.0, bs = 0.0;
    // the filter's M2 terms and the fs_in state loaded with the first chunk (one record
    // round trip when nb <= LREC: the second pass reuses the first's loads)
    double rn1[LREC], rm1[LREC], rs1[LREC];
    const double n0 = fs_in[isr ? 1 : 0], M0 = fs_in[2 + k], S0 = fs_in[2 + D + k];
    if (a.nb <= LREC) {
#pragma unroll
      for (int q = 0; q < LREC; ++q) {
        const double* r = rec + (int64_t)min(q, a.nb - 1) * a.RS;
        rn1[q] = r[isr ? 1 : 0];
        rm1[q] = r[2 + k];
        rs1[q] = r[2 + D + k];
      }
#pragma unroll
      for (int q = 0; q < LREC; ++q)
        if (q < a.nb) {
          bn += rn1[q];
          sm += rn1[q] * rm1[q];
        }
      if (bn > 0.0) {
        bm = sm / bn;
#pragma unroll
        for (int q = 0; q < LREC; ++q)
          if (q < a.nb && rn1[q] > 0.0) {
            const double dm = rm1[q] - bm;
            bs += rs1[q] + rn1[q] * dm * dm;
          }
      }
    } else {
      for (int b0 = 0; b0 < a.nb; b0 += LREC) {
        double rn[LREC], rm[LREC];
#pragma unroll
        for (int q = 0; q < LREC; ++q) {
          const double* r = rec + (int64_t)min(b0 + q, a.nb - 1) * a.RS;
          rn[q] = r[isr ? 1 : 0];
          rm[q] = r[2 + k];
        }
#pragma unroll
        for (int q = 0; q < LREC; ++q)
          if (b0 + q < a.nb) {
            bn += rn[q];
            sm += rn[q] * rm[q];
          }
      }
      if (bn > 0.0) {
        bm = sm / bn;
        for (int b0 = 0; b0 < a.nb; b0 += LREC) {
          double rn[LREC], rm[LREC], rs[LREC];
#pragma unroll
          for (int q = 0; q < LREC; ++q) {
            const double* r = rec + (int64_t)min(b0 + q, a.nb - 1) * a.RS;
            rn[q] = r[isr ? 1 : 0];
            rm[q] = r[2 + k];
            rs[q] = r[2 + D + k];
          }
#pragma unroll
          for (int q = 0; q < LREC; ++q)
            if (b0 + q < a.nb && rn[q] > 0.0) {
              const double dm = rm[q] - bm;
              bs += rs[q] + rn[q] * dm * dm;
            }
        }
      }
    }
    double n = n0, M = M0, S = S0;
    chan_merge(n, M, S, bn, bm, bs);
    if (blockIdx.x == 0) {
      if (k == 0) fs_out[0] = n;
      if (isr) fs_out[1] = n;
      fs_out[2 + k] = M;
      fs_out[2 + D + k] = S;
    }
    const double var = n > 1.0 ? S / (n - 1.0) : M * M;  // running_stat.py:27
    fmean[threadIdx.x] = M;
    fden[threadIdx.x] = sqrt(var) + 1e-8;
  }
  __syncthreads();
  // normalised obs rows (core.py:191-192): SoA raw -> LDS tile -> row-major fp32 rows
  const int64_t row0 = (int64_t)t * E + e0;
  {
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      const int kl = kb + G * q;
      double x = v[q];
      if (a.d.filter) {
        x = x - fmean[kl];
        x = x / fden[kl];
        x = x < -5.0 ? -5.0 : (x > 5.0 ? 5.0 : x);
      }
      tile[kl * (ENVS_PER_BLOCK + 1) + el] = (float)x;
    }
  }
  __syncthreads();
  {
    const int el = threadIdx.x / G, part = threadIdx.x % G;
    if (el < nvalid) {
      float* dst = a.b.obs + (row0 + el) * O;
      // the bf16 twin of the row for the first hidden GEMM (mrl_cast_rows_bf16's RNE)
      uint16_t* dsb = a.b.obs_bf16 ? a.b.obs_bf16 + (int64_t)(e0 + el) * ((O + 7) / 8 * 8) : nullptr;
#pragma unroll
      for (int q = 0; q < CPT; ++q) {
        const int k = kbase + part * CPT + q;
        const float v = tile[(part * CPT + q) * (ENVS_PER_BLOCK + 1) + el];
        if (k < O) {
          dst[k] = v;
          if (dsb) dsb[k] = __builtin_bit_cast(uint16_t, (__bf16)v);
        }
      }
    }
  }
}

// sample + env step + raw next obs / reward (SoA) for one env per thread
template <int ENV>
__global__ __launch_bounds__(RB) void lrollout_act_kernel(RollArgs a, const float* __restrict__ zrows,
                                                          const float* __restrict__ logstd, int t) {
  using EC = EnvC<ENV>;
  constexpr int O = EC::OBS, NS = EC::NS, A = EC::ACT;
  const int E = a.d.n_envs;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t row = (int64_t)t * E + e;
  double s[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) s[i] = a.b.env_state[(int64_t)i * E + e];
  float z[A];
#pragma unroll
  for (int q = 0; q < A; ++q) z[q] = zrows[(int64_t)e * A + q];
  double zn[A + 1];
  load_noise<ENV>(a, row, zn);
  double rew = 0.0;
  bool done = false;
  sample_and_step<ENV>(a, row, z, logstd, zn, s, rew, done);
  finish_env_step<ENV>(a, e, row, t, s, rew, done);
  double* raw = a.b.raw_obs;
  EC::obs_out(s, [&](int k, double v) { raw[(int64_t)k * E + e] = v; });
  raw[(int64_t)O * E + e] = rew;
}

// Humanoid-v2 on the layered rollout: one wave per env (humanoid.h), its state in LDS.
// hm_reset_kernel = lrollout_reset_kernel, hm_act_kernel = lrollout_act_kernel.
// WPB waves (envs) per block: 1 -- a one-wave block per env, padded so that at most four
// share a CU (hm_lds_pad) -- or 4 -- four envs per block sharing one copy of the model
// tables (94 KB of LDS, so one block per CU; the LDS left beside it takes a co-scheduled
// kernel's blocks without displacing an env).  Waves are independent after the tables'
// barrier (a wave's LDS operations complete in issue order).
// The tables and (WPB = 1) the env's state are static LDS objects -- their addresses are
// constants the ds instructions take as offsets; the WPB = 4 states sit in dynamic LDS
// after them, one wave-uniform base each.
template <int WPB>
__device__ inline hm::Wave& hm_block(int& e, int& lane) {
  extern __shared__ __attribute__((aligned(16))) double hm_dyn[];
  lane = threadIdx.x & 63;
  if constexpr (WPB == 1) {
    __shared__ hm::Wave W1;
    e = blockIdx.x;
    return W1;
  } else {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e = blockIdx.x * WPB + wave;
    return reinterpret_cast<hm::Wave*>(hm_dyn)[wave];
  }
}
template <int WPB>
__device__ inline void hm_load_tables(hm::Shared& S, int lane) {
  if (WPB == 1) {
    hm::load_shared(S, lane);
  } else {  // the block's waves copy disjoint parts, then wait for each other
    const double* src = reinterpret_cast<const double*>(&hm::SHARED);
    double* dst = reinterpret_cast<double*>(&S);
    for (int i = threadIdx.x; i < (int)(sizeof(hm::Shared) / 8); i += 64 * WPB) dst[i] = src[i];
    __syncthreads();
  }
}

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void hm_reset_kernel(RollArgs a) {
  __shared__ hm::Shared S;
  int e, lane;
  hm::Wave& W = hm_block<WPB>(e, lane);
  const int E = a.d.n_envs;
  hm_load_tables<WPB>(S, lane);
  if (e >= E) return;  // after the tables' barrier
  const uint32_t w = (uint32_t)a.b.env_int[E + e];
  hm::reset(W, lane, a.d.seed, (uint32_t)(a.d.env_offset + e), (uint64_t)w);
  hm::forward(W, S, lane);
  double* raw = a.b.raw_obs;
  hm::observation(W, S, lane, [&](int k, double v) { raw[(int64_t)k * E + e] = v; });
  if (lane < HM_NS) a.b.env_state[(int64_t)lane * E + e] = W.s[lane];
  hm::save_kcache(W, a.b.env_state + (int64_t)HM_NS * E + (int64_t)e * HM_KCACHE, lane);
  if (lane == 0) {
    raw[(int64_t)HM_OBS * E + e] = 0.0;
    a.b.env_int[E + e] = (int32_t)(w + 1);
    a.b.env_int[e] = 0;
  }
}

// The policy head fused into the step (HeadRows.hid != nullptr): z = hid[e] . W + b for
// the env's row of the last hidden layer, lane-strided over the hidden units (17
// accumulators per lane) and reduced across the wave in a fixed order -- one launch of
// a 1024 x 512 x 17 GEMM with 8 blocks (33 us per step) removed.  bf: the operands
// rounded to bf16 like the layered bf16 GEMM's (products and sums stay f32).
struct HeadRows {
  const float* hid;  // [E, nh] rows of the last hidden layer, or nullptr: z rows given
  const float* w;    // [nh, A] head kernel (Keras layout)
  const float* b;    // [A]
  int nh, bf;
  const uint16_t* hid16;  // the hidden rows as bf16 bits instead of hid (the bf16 tape's)
};

// lane l takes the KPL consecutive hidden units KPL l .. KPL l + KPL - 1: their head-kernel
// rows are one contiguous, 16-B aligned run of KPL A floats (KPL % 4 == 0), loaded as
// float4s -- a quarter of the strided lane-per-unit loads' instructions (nh = 64 KPL)
template <int KPL>
__device__ inline float head_z_runs(const HeadRows& hr, int e, int lane) {
  constexpr int A = HM_ACT;
  static_assert(KPL % 4 == 0, "16-B aligned runs");
  float acc[A], hv[KPL];
#pragma unroll
  for (int o = 0; o < A; ++o) acc[o] = 0.f;
  if (hr.hid16) {
    const uint4* h = reinterpret_cast<const uint4*>(hr.hid16 + (int64_t)e * hr.nh + KPL * lane);
#pragma unroll
    for (int q = 0; q < KPL / 8; ++q) {
      const uint4 u = h[q];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[8 * q + 2 * r] = __uint_as_float(w[r] << 16);
        hv[8 * q + 2 * r + 1] = __uint_as_float(w[r] & 0xffff0000u);
      }
    }
    if constexpr (KPL % 8 != 0) {
      const uint2 u = reinterpret_cast<const uint2*>(hr.hid16 + (int64_t)e * hr.nh + KPL * lane)[KPL / 4 - 1];
      hv[KPL - 4] = __uint_as_float(u.x << 16);
      hv[KPL - 3] = __uint_as_float(u.x & 0xffff0000u);
      hv[KPL - 2] = __uint_as_float(u.y << 16);
      hv[KPL - 1] = __uint_as_float(u.y & 0xffff0000u);
    }
  } else {
    const float4* h = reinterpret_cast<const float4*>(hr.hid + (int64_t)e * hr.nh + KPL * lane);
#pragma unroll
    for (int q = 0; q < KPL / 4; ++q) {
      const float4 u = h[q];
      hv[4 * q] = hr.bf ? bf16r(u.x) : u.x;
      hv[4 * q + 1] = hr.bf ? bf16r(u.y) : u.y;
      hv[4 * q + 2] = hr.bf ? bf16r(u.z) : u.z;
      hv[4 * q + 3] = hr.bf ? bf16r(u.w) : u.w;
    }
  }
  const float4* w4 = reinterpret_cast<const float4*>(hr.w + (int64_t)KPL * lane * A);
#pragma unroll
  for (int q = 0; q < KPL * A / 4; ++q) {
    const float4 w = w4[q];
    const float ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 4 * q + r;
      acc[f % A] = fmaf(hv[f / A], hr.bf ? bf16r(ws[r]) : ws[r], acc[f % A]);
    }
  }
  float z = 0.f;
#pragma unroll
  for (int o = 0; o < A; ++o) {
    const float sum = wave_sumf(acc[o]);
    if (lane == o) z = sum + hr.b[o];
  }
  return z;
}

__device__ inline float head_z(const HeadRows& hr, int e, int lane) {
  constexpr int A = HM_ACT;
  const bool al = (reinterpret_cast<uintptr_t>(hr.w) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(hr.hid16 ? (const void*)hr.hid16 : (const void*)hr.hid) & 15) == 0;
  if (al && hr.nh == 512) return head_z_runs<8>(hr, e, lane);
  if (al && hr.nh == 256) return head_z_runs<4>(hr, e, lane);
  float acc[A];
#pragma unroll
  for (int o = 0; o < A; ++o) acc[o] = 0.f;
  const float* hrow = hr.hid + (int64_t)e * hr.nh;
  const uint16_t* hrow16 = hr.hid16 + (int64_t)e * hr.nh;
  for (int k = lane; k < hr.nh; k += 64) {
    const float hv = hr.hid16 ? __uint_as_float((uint32_t)hrow16[k] << 16) : (hr.bf ? bf16r(hrow[k]) : hrow[k]);
    const float* wr = hr.w + (int64_t)k * A;
#pragma unroll
    for (int o = 0; o < A; ++o) acc[o] = fmaf(hv, hr.bf ? bf16r(wr[o]) : wr[o], acc[o]);
  }
  float z = 0.f;
#pragma unroll
  for (int o = 0; o < A; ++o) {
    const float sum = wave_sumf(acc[o]);
    if (lane == o) z = sum + hr.b[o];
  }
  return z;
}

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void hm_act_kernel(RollArgs a, const float* __restrict__ zrows, HeadRows hr,
                                                          const float* __restrict__ logstd, int t) {
  __shared__ hm::Shared S;
  int e, lane;
  hm::Wave& W = hm_block<WPB>(e, lane);
  constexpr int A = HM_ACT;
  const int E = a.d.n_envs;
  const bool live = e < E;
  const int ec = live ? e : E - 1;  // a block's waves past E load a valid env, store nothing
  double* const kc = a.b.env_state + (int64_t)HM_NS * E + (int64_t)ec * HM_KCACHE;
  const bool fused = hr.hid != nullptr || hr.hid16 != nullptr;
  float zh = 0.f;
  if constexpr (WPB == 4) {
    // the model tables' global loads first, held in registers while the env's own loads
    // (state, kinematics cache) and the head's dot products run, stored behind them:
    // one load latency for the launch's prologue instead of three in sequence
    constexpr int NW = (int)(sizeof(hm::Shared) / 8), PER = (NW + 64 * WPB - 1) / (64 * WPB);
    const double* src = reinterpret_cast<const double*>(&hm::SHARED);
    double tv[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = (int)threadIdx.x + 64 * WPB * i;
      tv[i] = src[k < NW ? k : 0];
    }
    if (lane < HM_NS) W.s[lane] = a.b.env_state[(int64_t)lane * E + ec];
    hm::load_kcache(W, kc, lane);
    if (fused) zh = head_z(hr, ec, lane);
    double* dst = reinterpret_cast<double*>(&S);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = (int)threadIdx.x + 64 * WPB * i;
      if (k < NW) dst[k] = tv[i];
    }
    __syncthreads();
  } else {
    hm_load_tables<WPB>(S, lane);
    if (lane < HM_NS) W.s[lane] = a.b.env_state[(int64_t)lane * E + ec];
    hm::load_kcache(W, kc, lane);
    if (fused) zh = head_z(hr, ec, lane);
  }
  if (!live) return;  // after the tables' barrier
  const int64_t row = (int64_t)t * E + e;
  WAVE_SYNC();
  // sample (DiagGauss, core.py:432-435): a = z + sd * noise in fp32; the action is the ctrl
  if (lane < A) {
    const float z = fused ? zh : zrows[(int64_t)e * A + lane];
    const float sd = expf(logstd[lane]);
    const double zn = reinterpret_cast<const double*>(a.b.noise)[row * A + lane];
    const float av = __fadd_rn(__fmul_rn((float)zn, sd), z);
    reinterpret_cast<float*>(a.b.act)[row * A + lane] = av;
    a.b.prob[row * 2 * A + lane] = z;
    a.b.prob[row * 2 * A + A + lane] = sd;
    W.s[HM_NQ + HM_NV + lane] = (double)av;
  }
  WAVE_SYNC();
  // one forward site (the kernel's code must fit the instruction cache): passes
  // 0..FRAME_SKIP-1 are the substeps, pass FRAME_SKIP observes the new state, pass
  // FRAME_SKIP + 1 the reset one
  double x_before = 0.0, rew = 0.0;
  // diagnostic stamps of block 0 (cols 0-11: phases of pass 1, 12/15 realtime and
  // 13/14 shader clock at kernel start / end) -- never set in production
  int64_t* st = (a.b.stamps != nullptr && e == 0) ? a.b.stamps + (int64_t)t * 16 : nullptr;
  if (st != nullptr && lane == 0) {
    st[12] = (int64_t)__builtin_amdgcn_s_memrealtime();
    st[13] = (int64_t)__builtin_amdgcn_s_memtime();
  }
  for (int pass = 0;; ++pass) {
    int64_t* sp = pass == 1 ? st : nullptr;
    if (sp != nullptr && lane == 0) sp[0] = (int64_t)__builtin_amdgcn_s_memtime();
    if (pass > 0) hm::forward(W, S, lane, sp);  // pass 0: the kinematics cache
    if (pass < hm::FRAME_SKIP) {
      if (pass == 0) x_before = W.com[0];
      hm::accelerations(W, S, lane, sp);
      hm::integrate(W, lane);
      continue;
    }
    if (pass > hm::FRAME_SKIP) break;
    bool done;
    hm::reward_done(W, lane, x_before, rew, done);
    // episode bookkeeping (finish_env_step): TimeLimit => terminated, limit / horizon cut => not
    const int ept = a.b.env_int[e];
    const bool term = done || (ept + 1 >= EnvC<MRL_ENV_HUMANOID>::MAX_STEPS);
    const bool last = term || (ept + 1 >= a.d.timestep_limit) || (t == a.d.horizon - 1);
    if (lane == 0) {
      a.b.ep_t[row] = ept;
      a.b.rew[row] = (float)rew;
      a.b.flags[row] = (uint8_t)((last ? 1 : 0) | (term ? 2 : 0));
    }
    if (!(last && t < a.d.horizon - 1)) {
      if (lane == 0) a.b.env_int[e] = ept + 1;
      break;
    }
    const uint32_t w = (uint32_t)a.b.env_int[E + e];
    hm::reset(W, lane, a.d.seed, (uint32_t)(a.d.env_offset + e), (uint64_t)w);
    if (lane == 0) {
      a.b.env_int[E + e] = (int32_t)(w + 1);
      a.b.env_int[e] = 0;
    }
  }
  if (lane < HM_NS) a.b.env_state[(int64_t)lane * E + e] = W.s[lane];
  hm::save_kcache(W, kc, lane);  // W holds forward() of the state just stored
  double* raw = a.b.raw_obs;
  hm::observation(W, S, lane, [&](int k, double v) { raw[(int64_t)k * E + e] = v; });
  if (lane == 0) raw[(int64_t)HM_OBS * E + e] = rew;
  if (st != nullptr && lane == 0) {
    st[14] = (int64_t)__builtin_amdgcn_s_memtime();
    st[15] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
}

// Dynamic LDS padding for the wave-per-env Humanoid step: while the envs fit one wave
// per SIMD, at most 4 blocks (waves) may share a CU, so the dispatcher cannot stack two
// latency chains on one SIMD and leave another idle.
static size_t hm_lds_pad(int n_envs) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      ncu = n;
    else
      ncu = -1;
  }
  if (ncu <= 0 || n_envs > 4 * ncu) return 0;
  constexpr size_t LDS_CU = 160 * 1024, used = sizeof(hm::Wave) + sizeof(hm::Shared), want = LDS_CU / 5 + 1024;
  return used < want ? want - used : 0;
}
// MRL_HM_WPB (per launch): four envs per block (hm_block, the default) or 1
static int hm_wpb() {
  // r04i (C5 bf16, 1024 envs): the rollout alone 225 -> 212 ms per iteration, beside the
  // co-scheduled fit 269 -> 260 ms (one table copy per four envs, 94 KB of LDS per CU)
  const char* e = getenv("MRL_HM_WPB");
  return (e && atoi(e) == 1) ? 1 : 4;
}
// dynamic LDS of a launch (the static tables / state come on top)
static size_t hm_lds_bytes(int wpb, int n_envs) {
  return wpb == 1 ? hm_lds_pad(n_envs) : (size_t)wpb * sizeof(hm::Wave);
}

__global__ void rollout_finish_kernel(RollArgs a, int O) {
  const int D = O + 1, T = a.d.horizon;
  const double* fs_in = a.b.filter_state + (T & 1) * a.FS;
  double* fs_out = a.b.filter_state;
  const double* rec_in = a.b.records + (int64_t)(T & 1) * a.nb * a.RS;
  const int g = threadIdx.x >> 4, j = threadIdx.x & 15;
  // the last step's rewards still go through rewfilt (core.py:199); obs_T is never pushed
  double n = 0.0, M = 0.0, S = 0.0;
  if (g == 0) {
    n = fs_in[1];
    M = fs_in[2 + O];
    S = fs_in[2 + D + O];
    double bn, bm, bs;
    batch_of_records(rec_in, a.nb, a.RS, D, O, O, j, bn, bm, bs);
    chan_merge(n, M, S, bn, bm, bs);
  }
  // copy the obs stat when fs_in is the other buffer (T odd)
  double cp[(MAXD_L + RB - 1) / RB * 2 + 1];
  int nc = 0;
  if ((T & 1) != 0)
    for (int k = threadIdx.x; k < O; k += RB) {
      cp[nc++] = fs_in[2 + k];
      cp[nc++] = fs_in[2 + D + k];
    }
  const double n_obs = fs_in[0];
  __syncthreads();  // fs_in may alias fs_out (T even)
  if ((T & 1) != 0) {
    nc = 0;
    for (int k = threadIdx.x; k < O; k += RB) {
      fs_out[2 + k] = cp[nc++];
      fs_out[2 + D + k] = cp[nc++];
    }
    if (threadIdx.x == 0) fs_out[0] = n_obs;
  }
  if (g == 0 && j == 0) {
    fs_out[1] = n;
    fs_out[2 + O] = M;
    fs_out[2 + D + O] = S;
  }
  if (threadIdx.x == 0) *a.b.iteration += 1;
}

}  // namespace mrl

using namespace mrl;

static int check_roll(const mrl_rollout_desc* d, const mrl_rollout_bufs* b) {
  if (!d || !b) return fail(E_ARG, "null desc/bufs");
  if (d->env_id != MRL_ENV_CARTPOLE && d->env_id != MRL_ENV_HOPPER && d->env_id != MRL_ENV_HUMANOID)
    return fail(E_UNSUPPORTED, "unknown env_id");
  if (d->n_envs <= 0 || d->horizon <= 0 || d->timestep_limit <= 0) return fail(E_ARG, "bad sizes");
  if (d->compute != MRL_COMPUTE_F32 && d->compute != MRL_COMPUTE_BF16) return fail(E_ARG, "bad compute");
  if (!b->env_state || !b->env_int || !b->filter_state || !b->records || !b->iteration) return fail(E_ARG, "null state");
  return OK;
}

static RollArgs make_args(const mrl_rollout_desc* d, const mrl_rollout_bufs* b) {
  RollArgs a;
  a.d = *d;
  a.b = *b;
  a.nb = (d->n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  a.FS = filt_doubles(env_info(d->env_id).obs);
  a.RS = a.FS;
  return a;
}

#define MRL_DISPATCH_ENV(id, KERNEL, ...)                                                    \
  do {                                                                                      \
    if ((id) == MRL_ENV_CARTPOLE) hipLaunchKernelGGL(KERNEL<MRL_ENV_CARTPOLE>, __VA_ARGS__); \
    else if ((id) == MRL_ENV_HOPPER) hipLaunchKernelGGL(KERNEL<MRL_ENV_HOPPER>, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<MRL_ENV_HUMANOID>, __VA_ARGS__);                         \
  } while (0)

extern "C" {

// Humanoid: the state (SoA [NS][E]) and then each env's kinematics cache (AoS [E][KCACHE],
// humanoid.h save_kcache) -- the forward kinematics of the stored state
int64_t mrl_env_state_doubles(int32_t env_id) {
  return env_info(env_id).ns + (env_id == MRL_ENV_HUMANOID ? HM_KCACHE : 0);
}
int64_t mrl_filter_doubles(int32_t env_id) { return filt_doubles(env_info(env_id).obs); }
int64_t mrl_record_doubles(int32_t env_id) { return filt_doubles(env_info(env_id).obs); }
int64_t mrl_rollout_blocks(int32_t n_envs) { return (n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK; }
int64_t mrl_rollout_noise_doubles(const mrl_rollout_desc* d) {
  if (!d || d->n_envs <= 0 || d->horizon <= 0) return -1;
  const EnvInfo ei = env_info(d->env_id);
  return (int64_t)d->horizon * d->n_envs * (ei.discrete ? 1 : ei.act);
}

int mrl_rollout_noise(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, double* out, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (!out) return fail(E_ARG, "null noise rows");
  RollArgs a = make_args(d, b);
  const EnvInfo ei = env_info(d->env_id);
  const int64_t per_step = (int64_t)d->n_envs * (ei.discrete ? 1 : (ei.act + 1) / 2);
  MRL_DISPATCH_ENV(d->env_id, noise_fill_kernel, dim3((unsigned)((per_step + 255) / 256), (unsigned)(d->horizon < 65535 ? d->horizon : 65535)),
                   dim3(256), 0, (hipStream_t)stream, a, out);
  return hip_check(hipGetLastError(), "mrl_rollout_noise");
}

int mrl_rollout_reset(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (d->env_id == MRL_ENV_HUMANOID) return fail(E_UNSUPPORTED, "Humanoid runs on the layered rollout (mrl_rollout_reset_rows)");
  RollArgs a = make_args(d, b);
  if (d->env_id == MRL_ENV_CARTPOLE)
    hipLaunchKernelGGL(rollout_reset_kernel<MRL_ENV_CARTPOLE>, dim3(a.nb), dim3(RB), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(rollout_reset_kernel<MRL_ENV_HOPPER>, dim3(a.nb), dim3(RB), 0, (hipStream_t)stream, a);
  return hip_check(hipGetLastError(), "mrl_rollout_reset");
}


static int check_rows(const mrl_rollout_desc* d, const mrl_rollout_bufs* b) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (!b->raw_obs) return fail(E_ARG, "the layered rollout needs raw_obs [(obs_dim+1) * n_envs] doubles");
  if (env_info(d->env_id).obs + 1 > MAXD_L) return fail(E_UNSUPPORTED, "obs dim too large");
  return OK;
}

int mrl_rollout_reset_rows(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream) {
  int rc = check_rows(d, b);
  if (rc) return rc;
  RollArgs a = make_args(d, b);
  const int D = env_info(d->env_id).obs + 1;
  // one wave per block: the per-env step is latency-bound, so spread the waves over CUs
  const dim3 genv((d->n_envs + 63) / 64), gpart(a.nb, (D + LCOLS - 1) / LCOLS);
  if (d->env_id == MRL_ENV_HUMANOID) {
    const int wpb = hm_wpb();
    const dim3 gb((d->n_envs + wpb - 1) / wpb), bb(64 * wpb);
    const size_t lds = wpb == 1 ? 0 : (size_t)wpb * sizeof(hm::Wave);
    if (wpb == 4) hipLaunchKernelGGL(hm_reset_kernel<4>, gb, bb, lds, (hipStream_t)stream, a);
    else hipLaunchKernelGGL(hm_reset_kernel<1>, gb, bb, lds, (hipStream_t)stream, a);
  } else if (d->env_id == MRL_ENV_CARTPOLE)
    hipLaunchKernelGGL(lrollout_reset_kernel<MRL_ENV_CARTPOLE>, genv, dim3(64), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(lrollout_reset_kernel<MRL_ENV_HOPPER>, genv, dim3(64), 0, (hipStream_t)stream, a);
  hipLaunchKernelGGL(lrollout_partials_kernel, gpart, dim3(RB), 0, (hipStream_t)stream, a, D, 0, 0);
  return hip_check(hipGetLastError(), "mrl_rollout_reset_rows");
}

int mrl_rollout_obs(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, int32_t t, void* stream) {
  int rc = check_rows(d, b);
  if (rc) return rc;
  if (!b->obs) return fail(E_ARG, "null obs");
  if (t < 0 || t >= d->horizon) return fail(E_ARG, "t out of range");
  RollArgs a = make_args(d, b);
  const dim3 grid(a.nb, (env_info(d->env_id).obs + 1 + LCOLS - 1) / LCOLS);
  MRL_DISPATCH_ENV(d->env_id, lrollout_obs_kernel, grid, dim3(RB), 0, (hipStream_t)stream, a, t);
  return hip_check(hipGetLastError(), "mrl_rollout_obs");
}

static int rollout_act(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const float* z, const HeadRows& hr,
                       const float* logstd, const mrl_rollout_bufs* b, int32_t t, void* stream) {
  int rc = check_rows(d, b);
  if (rc) return rc;
  if (!b->act || !b->prob || !b->rew || !b->flags || !b->ep_t || (!z && !hr.hid && !hr.hid16))
    return fail(E_ARG, "null trajectory buffer");
  if ((hr.hid || hr.hid16) && d->env_id != MRL_ENV_HUMANOID)
    return fail(E_UNSUPPORTED, "the fused head is the Humanoid step's");
  if (!b->noise) return fail(E_ARG, "bufs.noise: sampling-noise rows (mrl_rollout_noise or injected) required");
  EnvInfo ei = env_info(d->env_id);
  const bool gauss = head == MRL_HEAD_GAUSS;
  if (n_out != ei.act || gauss == (bool)ei.discrete || (!gauss && head != MRL_HEAD_SOFTMAX))
    return fail(E_ARG, "policy head does not match the env");
  if (gauss && !logstd) return fail(E_ARG, "DiagGauss needs logstd");
  if (t < 0 || t >= d->horizon) return fail(E_ARG, "t out of range");
  RollArgs a = make_args(d, b);
  const int D = ei.obs + 1;
  const dim3 genv((d->n_envs + 63) / 64), gpart(a.nb, (D + LCOLS - 1) / LCOLS);
  if (d->env_id == MRL_ENV_HUMANOID) {
    const int wpb = hm_wpb();
    const dim3 gb((d->n_envs + wpb - 1) / wpb), bb(64 * wpb);
    const size_t lds = hm_lds_bytes(wpb, d->n_envs);
    if (wpb == 4) hipLaunchKernelGGL(hm_act_kernel<4>, gb, bb, lds, (hipStream_t)stream, a, z, hr, logstd, t);
    else hipLaunchKernelGGL(hm_act_kernel<1>, gb, bb, lds, (hipStream_t)stream, a, z, hr, logstd, t);
  } else if (d->env_id == MRL_ENV_CARTPOLE)
    hipLaunchKernelGGL(lrollout_act_kernel<MRL_ENV_CARTPOLE>, genv, dim3(64), 0, (hipStream_t)stream, a, z, logstd, t);
  else
    hipLaunchKernelGGL(lrollout_act_kernel<MRL_ENV_HOPPER>, genv, dim3(64), 0, (hipStream_t)stream, a, z, logstd, t);
  hipLaunchKernelGGL(lrollout_partials_kernel, gpart, dim3(RB), 0, (hipStream_t)stream, a, D, (t + 1) & 1, 1);
  return hip_check(hipGetLastError(), "mrl_rollout_act");
}

int mrl_rollout_act(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const float* z, const float* logstd,
                    const mrl_rollout_bufs* b, int32_t t, void* stream) {
  if (!z) return fail(E_ARG, "null z rows");
  return rollout_act(d, head, n_out, z, HeadRows{nullptr, nullptr, nullptr, 0, 0, nullptr}, logstd, b, t, stream);
}

int mrl_rollout_act_head(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const float* hidden,
                         int32_t n_hidden, const float* w_head, const float* b_head, const float* logstd,
                         const mrl_rollout_bufs* b, int32_t t, void* stream) {
  if (!d || !hidden || !w_head || !b_head || n_hidden <= 0) return fail(E_ARG, "mrl_rollout_act_head: bad arguments");
  if (d->env_id != MRL_ENV_HUMANOID || n_out != HM_ACT)
    return fail(E_UNSUPPORTED, "mrl_rollout_act_head: the fused head is the Humanoid step's (17 outputs)");
  return rollout_act(d, head, n_out, nullptr,
                     HeadRows{hidden, w_head, b_head, n_hidden, (int)(d->compute == MRL_COMPUTE_BF16), nullptr}, logstd,
                     b, t, stream);
}

int mrl_rollout_act_head_bf16(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const uint16_t* hidden16,
                              int32_t n_hidden, const float* w_head, const float* b_head, const float* logstd,
                              const mrl_rollout_bufs* b, int32_t t, void* stream) {
  if (!d || !hidden16 || !w_head || !b_head || n_hidden <= 0)
    return fail(E_ARG, "mrl_rollout_act_head_bf16: bad arguments");
  if (d->env_id != MRL_ENV_HUMANOID || n_out != HM_ACT)
    return fail(E_UNSUPPORTED, "mrl_rollout_act_head_bf16: the fused head is the Humanoid step's (17 outputs)");
  if (d->compute != MRL_COMPUTE_BF16) return fail(E_ARG, "mrl_rollout_act_head_bf16: bf16 hidden rows need MRL_COMPUTE_BF16");
  return rollout_act(d, head, n_out, nullptr, HeadRows{nullptr, w_head, b_head, n_hidden, 1, hidden16}, logstd, b, t,
                     stream);
}

static int check_fused_policy(const mrl_rollout_desc* d, const mrl_mlp_desc* pol) {
  EnvInfo ei = env_info(d->env_id);
  const bool gauss = pol->head == MRL_HEAD_GAUSS;
  if (pol->n_in != ei.obs || pol->n_out != ei.act || gauss == (bool)ei.discrete || pol->n_hidden != HID ||
      pol->n_layers != 2)
    return fail(E_ARG, "policy shape does not match the env");
  return OK;
}

int64_t mrl_rollout_image_floats(const mrl_mlp_desc* pol) {
  if (!pol || pol->n_in <= 0 || pol->n_in > MAX_IN) return -1;
  return rollout_dims(pol->n_in).size;
}

int mrl_rollout_pack(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, float* rimage,
                     void* stream) {
  if (!d || !pol || !theta || !rimage) return fail(E_ARG, "null pointer");
  if (d->env_id == MRL_ENV_HUMANOID) return fail(E_UNSUPPORTED, "Humanoid runs on the layered rollout");
  int rc = check_fused_policy(d, pol);
  if (rc) return rc;
  const RDims r = rollout_dims(pol->n_in);
  const MlpDims md = mlp_dims(pol->n_in, pol->n_out, pol->head == MRL_HEAD_GAUSS);
  hipLaunchKernelGGL(rollout_pack_kernel, dim3((r.size + 255) / 256), dim3(256), 0, (hipStream_t)stream, r, md, theta,
                     rimage, (int)(d->compute == MRL_COMPUTE_BF16));
  return hip_check(hipGetLastError(), "mrl_rollout_pack");
}

int64_t mrl_rollout_sync_bytes(const mrl_rollout_desc* d) {
  if (!d || d->n_envs <= 0) return -1;
  const int64_t nb = (d->n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  return SYNC_HEAD_BYTES + 2 * (int64_t)(env_info(d->env_id).obs + 1) * nb * 16;
}

// Zeroes the hand-off workspace before a persistent launch (plain 16-B vector stores;
// the kernel boundary publishes them).  A kernel, not hipMemsetAsync: replayed from a
// captured hipGraph after other work had been launched eagerly, the memset node of
// ROCm 7.2 wrote a repeated 16-B pattern -- {int64 n, double 1/n}, bytes of a later
// eager launch's arguments -- instead of zeros (tools/dbg/sync_probe.py).
__global__ __launch_bounds__(256) void sync_clear_kernel(uint4* __restrict__ p, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

// The nb blocks fit one per CU of the launch stream (its CU mask) at this kernel's
// register use: the persistent launch may run (its blocks wait on each other, so the
// whole grid must be resident at once).  launch_cus > 0: the CUs of the stream a
// captured graph will replay on (the capture stream's mask says nothing about it);
// < 0: debug, no check.
static bool persistent_fits(int nb, hipStream_t s, int launch_cus) {
  if (launch_cus < 0) return true;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  int cus = ncu;
  if (s != nullptr) {
    uint32_t mask[16] = {};
    const int words = (ncu + 31) / 32;
    if (words <= 16 && hipExtStreamGetCUMask(s, (uint32_t)words, mask) == hipSuccess) {
      cus = 0;
      for (int w = 0; w < words; ++w) cus += __builtin_popcount(mask[w]);
    }
  }
  if (launch_cus > 0) cus = min(launch_cus, ncu);
  return nb <= cus;
}

int mrl_rollout_run(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, const float* rimage,
                    const mrl_rollout_bufs* b, uint32_t* sync, int32_t persistent, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (!pol || !theta || !rimage) return fail(E_ARG, "null policy");
  if (d->env_id == MRL_ENV_HUMANOID) return fail(E_UNSUPPORTED, "Humanoid runs on the layered rollout");
  if (!b->obs || !b->act || !b->prob || !b->rew || !b->flags || !b->ep_t) return fail(E_ARG, "null trajectory buffer");
  if (!b->noise) return fail(E_ARG, "bufs.noise: sampling-noise rows (mrl_rollout_noise or injected) required");
  rc = check_fused_policy(d, pol);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  RollArgs a = make_args(d, b);
  if (!persistent || !sync || !persistent_fits(a.nb, s, d->launch_cus)) {
    rc = mrl_rollout_reset(d, b, stream);
    for (int32_t t = 0; t < d->horizon && rc == OK; ++t) rc = mrl_rollout_step(d, pol, theta, rimage, b, t, stream);
    return rc;
  }
  const MlpDims md = mlp_dims(pol->n_in, pol->n_out, pol->head == MRL_HEAD_GAUSS);
  const float* logstd = pol->head == MRL_HEAD_GAUSS ? theta + md.tls : nullptr;
  {
    const int64_t n16 = mrl_rollout_sync_bytes(d) / 16;  // SYNC_HEAD_BYTES + 16-B granules
    const int nblk = (int)std::min<int64_t>((n16 + 255) / 256, 256);
    hipLaunchKernelGGL(sync_clear_kernel, dim3(nblk), dim3(256), 0, s, reinterpret_cast<uint4*>(sync), n16);
  }
  // A plain launch: persistent_fits() guarantees one block per CU of the stream's CU
  // set, so every block becomes resident (kernels of other streams on those CUs finish
  // on their own), and the step hand-off polls are bounded (SPIN_LIMIT).  A cooperative
  // launch made HIP keep a runtime-owned queue that its teardown destroyed after an
  // attached rocprofv3 had finalised: the profiled process crashed at exit.
  const bool bf = d->compute == MRL_COMPUTE_BF16, st = b->stamps != nullptr;
#define MRL_PERSIST(ENV, BF, ST) \
  hipLaunchKernelGGL((rollout_persistent_kernel<ENV, BF, ST>), dim3(a.nb), dim3(RB), 0, s, a, logstd, rimage, sync)
  if (d->env_id == MRL_ENV_CARTPOLE) {
    if (st && bf) MRL_PERSIST(MRL_ENV_CARTPOLE, true, true);
    else if (st) MRL_PERSIST(MRL_ENV_CARTPOLE, false, true);
    else if (bf) MRL_PERSIST(MRL_ENV_CARTPOLE, true, false);
    else MRL_PERSIST(MRL_ENV_CARTPOLE, false, false);
  } else {
    if (st && bf) MRL_PERSIST(MRL_ENV_HOPPER, true, true);
    else if (st) MRL_PERSIST(MRL_ENV_HOPPER, false, true);
    else if (bf) MRL_PERSIST(MRL_ENV_HOPPER, true, false);
    else MRL_PERSIST(MRL_ENV_HOPPER, false, false);
  }
#undef MRL_PERSIST
  return hip_check(hipGetLastError(), "mrl_rollout_run");
}

int mrl_rollout_step(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, const float* rimage,
                     const mrl_rollout_bufs* b, int32_t t, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (!pol || !theta || !rimage) return fail(E_ARG, "null policy");
  if (d->env_id == MRL_ENV_HUMANOID) return fail(E_UNSUPPORTED, "Humanoid runs on the layered rollout");
  if (!b->obs || !b->act || !b->prob || !b->rew || !b->flags || !b->ep_t) return fail(E_ARG, "null trajectory buffer");
  if (!b->noise) return fail(E_ARG, "bufs.noise: sampling-noise rows (mrl_rollout_noise or injected) required");
  rc = check_fused_policy(d, pol);
  if (rc) return rc;
  if (t < 0 || t >= d->horizon) return fail(E_ARG, "t out of range");
  RollArgs a = make_args(d, b);
  const MlpDims md = mlp_dims(pol->n_in, pol->n_out, pol->head == MRL_HEAD_GAUSS);
  const float* logstd = pol->head == MRL_HEAD_GAUSS ? theta + md.tls : nullptr;
  const bool bf = d->compute == MRL_COMPUTE_BF16;
  hipStream_t s = (hipStream_t)stream;
  if (d->env_id == MRL_ENV_CARTPOLE) {
    if (bf) hipLaunchKernelGGL((rollout_step_kernel<MRL_ENV_CARTPOLE, true>), dim3(a.nb), dim3(RB), 0, s, a, logstd, rimage, t);
    else hipLaunchKernelGGL((rollout_step_kernel<MRL_ENV_CARTPOLE, false>), dim3(a.nb), dim3(RB), 0, s, a, logstd, rimage, t);
  } else {
    if (bf) hipLaunchKernelGGL((rollout_step_kernel<MRL_ENV_HOPPER, true>), dim3(a.nb), dim3(RB), 0, s, a, logstd, rimage, t);
    else hipLaunchKernelGGL((rollout_step_kernel<MRL_ENV_HOPPER, false>), dim3(a.nb), dim3(RB), 0, s, a, logstd, rimage, t);
  }
  return hip_check(hipGetLastError(), "mrl_rollout_step");
}

int mrl_rollout_finish(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  RollArgs a = make_args(d, b);
  hipLaunchKernelGGL(rollout_finish_kernel, dim3(1), dim3(RB), 0, (hipStream_t)stream, a, env_info(d->env_id).obs);
  return hip_check(hipGetLastError(), "mrl_rollout_finish");
}

}  // extern "C"
