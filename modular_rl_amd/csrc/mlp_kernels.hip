// Fused MLP kernels of the TRPO hot path on v_mfma_f32_32x32x2_f32 (exact fp32).
//
//   mlp_rows_kernel<EPI>  forward (+ JVP) of a 32-row tile per wave with a per-row
//                         epilogue: prob rows, TRPO losses, surrogate gradient rows,
//                         VF loss rows, or the KL-metric rows of the Fisher product.
//   mlp_vjp_kernel        forward recompute + backprop of head-gradient rows and the
//                         weight-gradient sums  sum_rows act^T * grad  (MFMA with the
//                         row index as K, operands transposed through LDS).
//
// Replaces the Theano-compiled functions of the reference: _act_prob
// (core.py:269-270), compute_policy_gradient / compute_losses /
// compute_fisher_vector_product (trpo.py:68-70), NnRegression.predict and
// LbfgsOptimizer.f_lossgrad (core.py:608, 670-671).  The Fisher product uses the
// exact Gauss-Newton form of Theano's double backprop:
// JVP -> per-row KL metric -> VJP.
#include <math.h>

#include <stdlib.h>

#include <algorithm>

#include "../../include/mrl_hip.h"
#include "mlp_device.h"
#include "rows_epilogue.h"
#include "fvp_split_role.h"

namespace mrl {

static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
int fail(int code, const std::string& s) {
  g_err = s;
  return code;
}
int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return E_HIP;
  }
  return OK;
}

constexpr int ROWS_BLOCK = 256;
// The cached FVP rows kernel fits 3 blocks per CU (168 VGPRs, 2 x 23 KB images):
// 1536 = two full rounds of 768 resident blocks (1024 left a one-third second round;
// FVP rows 0.92 -> 0.90 ms at 4.19 M rows, the other rows kernels unchanged or faster)
#ifndef MRL_ROWS_MAX_BLOCKS
#define MRL_ROWS_MAX_BLOCKS 1536
#endif
constexpr int ROWS_MAX_BLOCKS = MRL_ROWS_MAX_BLOCKS;
constexpr int VJP_MAX_BLOCKS = 256;
constexpr int SCR_FLOATS = 2 * 64 * IMG_PAD;  // per-wave transpose scratch
#ifdef MRL_VJP_ABL_NOGW1  // diagnostic builds (tools/build_ablate.sh): drop one MFMA phase
#define VJP_ABL_S4 0
#else
#define VJP_ABL_S4 4
#endif

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int EPI_FVP_CACHED = 100;  // internal: MRL_EPI_FVP reading the activation cache

// the kernel arguments with a static shape's dimensions substituted (compile-time
// constants after inlining); SH == 0 leaves the run-time shape; SH | SH_TIME (mlp_layout.h)
// keeps ep_t for the time-feature column
template <int SH>
__device__ inline RowsArgs rows_shape(const RowsArgs& in) {
  RowsArgs a = in;
  if constexpr ((SH & ~SH_TIME) != 0) {
    constexpr int B = SH & ~SH_TIME;
    constexpr StaticShape S = STATIC_SHAPES[B];
    a.d = static_dims(B);
    a.A = S.A;
    a.head = S.head;
    a.n_obs = (SH & SH_TIME) ? S.O - 1 : S.O;
    a.gh = S.head == MRL_HEAD_GAUSS ? 2 * S.A : S.A;
    if constexpr (!(SH & SH_TIME)) a.ept = nullptr;
  }
  return a;
}

template <int EPI_K, int SH>
// 3 waves/SIMD: layer 2 is evaluated one M-tile at a time so the chain fits 168
// registers (the cached Fisher-product pass took 176 at a bound of 2, i.e. 2 waves)
__global__ __launch_bounds__(ROWS_BLOCK, 3) void mlp_rows_kernel(RowsArgs a_in, const float* __restrict__ img,
                                                               const float* __restrict__ imgt,
                                                               const int32_t* __restrict__ skip) {
  const RowsArgs a = rows_shape<SH>(a_in);
  constexpr bool CACHED = EPI_K == EPI_FVP_CACHED;
  constexpr int EPI = CACHED ? MRL_EPI_FVP : EPI_K;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const MlpDims& d = a.d;
  const int fs = d.fwd_size;
  for (int i = threadIdx.x; i < fs / 4; i += ROWS_BLOCK)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img)[i];
  if (EPI == MRL_EPI_FVP)
    for (int i = threadIdx.x; i < fs / 4; i += ROWS_BLOCK)
      reinterpret_cast<float4*>(lds + fs)[i] = reinterpret_cast<const float4*>(imgt)[i];
  __syncthreads();
  const float* ldt = lds + fs;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int A = a.A;
  float ls[MAX_OUT], sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
  for (int j = 0; j < MAX_OUT; ++j) {
    ls[j] = (a.logstd != nullptr && j < A) ? a.logstd[j] : 0.f;
    sd[j] = expf(ls[j]);
    dls[j] = (a.dlogstd != nullptr && j < A) ? a.dlogstd[j] : 0.f;
  }
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t row = tile * 32 + (lane & 31);
    const bool valid = row < a.n;
    XGlobal xl{a.x, a.ept, a.ts_limit, a.n_obs, row, valid};
    float z[MAX_OUT], dz[MAX_OUT];
    float* ctile = a.cache != nullptr ? a.cache + tile * CACHE_TILE_FLOATS : nullptr;
    if (CACHED) jvp_head_cached(lds, ldt, d, xl, lane, ctile, z, dz, a.head != MRL_HEAD_GAUSS);
    else if (EPI == MRL_EPI_FVP) forward_jvp_head_lowreg(lds, ldt, d, xl, lane, z, dz);
    else forward_head_lowreg(lds, d, xl, lane, z, a.cache_mode == MRL_CACHE_WRITE ? ctile : nullptr);
    if constexpr (EPI == MRL_EPI_PPOSGD) {
      // one 128-row minibatch per launch (ppo.py:150-156): block-reduced minibatch KL
      // sets the penalty slope, then the pensurr head gradient of every row
      __shared__ double red[4];
      if (valid && h == 0) row_epilogue<MRL_EPI_LOSSES, MAX_OUT>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
      const double klw = wave_sum(acc1);
      if (lane == 0) red[wave] = klw;
      __syncthreads();
      const double kl = ((red[0] + red[1]) + (red[2] + red[3])) * a.inv_ng;
      RowsArgs b = a;
      b.kl_coeff = a.kl_coeff + (kl > a.kl_cutoff ? (float)(2.0 * a.cutoff_coeff * (kl - a.kl_cutoff)) : 0.f);
      double d0 = 0.0, d1 = 0.0, d2 = 0.0;
      if (valid && h == 0) row_epilogue<MRL_EPI_PPOGRAD, MAX_OUT>(b, row, z, dz, ls, sd, dls, d0, d1, d2);
      continue;
    } else {
      if constexpr (EPI == MRL_EPI_PROB)
        if (a.feat != nullptr && valid) write_feature_row(a, row, h, xl);
      if (!valid || h != 0) continue;
      row_epilogue<EPI, MAX_OUT>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
    }
  }
  if (a.partial != nullptr) {
    acc0 = wave_sum(acc0);
    acc1 = wave_sum(acc1);
    acc2 = wave_sum(acc2);
    if (lane == 0) {
      double* p = a.partial + ((int64_t)blockIdx.x * 4 + wave) * 4;
      p[0] = acc0;
      p[1] = acc1;
      p[2] = acc2;
      p[3] = 0.0;
    }
  }
}

// ------------------------------------------------------------------ VJP
struct VjpArgs {
  MlpDims d;
  int n_obs, gh, n_sum;
  const float* x;
  const int32_t* ept;
  double ts_limit;
  int64_t n;
  const float* ghead;
  float* slab;
  const float* cache;  // primal activation cache (CACHED kernel)
};

// write a transposed tile (two 32x32 C tiles of 64 units) as img[unit][h'][s'],
// row j = 2 s' + h', per-unit stride IMG_PAD (conflict-free b32 writes, b128 reads)
__device__ inline void write_img(float* img, const f32x16* t, int lane) {
  const int j = lane & 31, h = lane >> 5;
  const int base = (j & 1) * 16 + (j >> 1);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) img[(32 * mt + cperm(r, h)) * IMG_PAD + base] = t[mt][r];
}


__device__ inline float rowsum32(const float* img, int unit) {
  const float* p = img + unit * IMG_PAD;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = ld4(p + 4 * q);
    s += (v.x + v.y) + (v.z + v.w);
  }
  return s;
}

// every global operand one tile needs, loaded ahead of use; CACHED: the primal
// activations come from the cache instead of the layer-0 inputs
// gW2 and gW0 run on v_mfma_f32_16x16x4_f32 (their narrow side -- A <= 8 head
// outputs, O <= 16 inputs per tile -- pads to 16 instead of 32).  Their K is the 32
// rows of the tile, read from the transposed LDS images at position p = 8*kk + q
// (kk = lane >> 4, k-step q), i.e. row r(p) = 16*(kk&1) + 2q + (kk>>1).
__device__ inline int vjp_row16(int kk, int q) { return 16 * (kk & 1) + 2 * q + (kk >> 1); }

template <bool CACHED, bool WIDE>
struct VjpIn {
  float x0[CACHED ? 1 : 16];  // layer-0 B operands x[row][2s+h]
  f32x16 act[CACHED ? 2 : 1]; // cached h2[0], h2[1] (h1 is loaded by the tile itself)
  float xg[WIDE ? 16 : 8];    // gW0 A operands x[row0 + r(8kk+q)][16mt + (lane&15)] at [8mt + q]
  float g[4];                 // head-gradient rows ghead[row][r+4h]
  float gs[MAX_OUT];          // summed head columns (DiagGauss logstd), lane half 0 only
};

// Branch-free loads: row indices are clamped to the batch and columns to the row
// width, so every load is unconditional straight-line code; what must read as zero
// (head-gradient entries of rows past n, of outputs past A, the logstd sums off lane
// half 0) is masked when the tile USES the values (a select at load time would force
// a wait right after the loads are issued).  The clamped gW0 operands of rows past
// n multiply head-gradient rows that are exactly zero; those of columns past the
// input width land in gW0 rows that are never stored.
// gW0 A operands of one tile (used last: issued after the operands of the first phases)
template <bool WIDE>
__device__ inline void vjp_load_xg(const VjpArgs& a, int64_t tile, int lane, float* xg) {
  const int i16 = lane & 15, kk = lane >> 4;
  constexpr int MT0 = WIDE ? 2 : 1;
  const int64_t row0 = tile * 32, last = a.n - 1;
  if (a.ept == nullptr) {
#pragma unroll
    for (int mt = 0; mt < MT0; ++mt) {
      const int c = 16 * mt + i16, cc = c < a.n_obs ? c : a.n_obs - 1;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t xr = row0 + vjp_row16(kk, q);
        xg[8 * mt + q] = a.x[(xr < last ? xr : last) * a.n_obs + cc];
      }
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < MT0; ++mt) {
      const int c = 16 * mt + i16;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t xr = row0 + vjp_row16(kk, q);
        XGlobal xq{a.x, a.ept, a.ts_limit, a.n_obs, xr, xr < a.n};
        xg[8 * mt + q] = (c < a.d.O) ? xq(c) : 0.f;
      }
    }
  }
}

template <bool CACHED, bool WIDE>
__device__ inline void vjp_load(const VjpArgs& a, int64_t tile, int lane, VjpIn<CACHED, WIDE>& in) {
  const int h = lane >> 5, j = lane & 31;
  const int64_t row0 = tile * 32, row = row0 + j, last = a.n - 1;
  if constexpr (CACHED) {
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
#pragma unroll
    for (int q = 0; q < 2; ++q) cache_load(ct, lane, 2 + q, in.act[q]);
  } else {
    XGlobal xl{a.x, a.ept, a.ts_limit, a.n_obs, row, row < a.n};
#pragma unroll
    for (int s = 0; s < 16; ++s) in.x0[s] = (s < a.d.KS0p) ? xl(2 * s + h) : 0.f;
  }
  const float* gr = a.ghead + (row < last ? row : last) * a.gh;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = r + 4 * h;
    in.g[r] = gr[o < a.gh ? o : a.gh - 1];
  }
#pragma unroll
  for (int q = 0; q < MAX_OUT; ++q) {
    const int c = a.d.A + q;
    in.gs[q] = gr[c < a.gh ? c : a.gh - 1];
  }
}

template <int SH>
__device__ inline VjpArgs vjp_shape(const VjpArgs& in) {
  VjpArgs a = in;
  if constexpr (SH != 0) {
    constexpr StaticShape S = STATIC_SHAPES[SH];
    a.d = static_dims(SH);
    a.n_obs = S.O;
    a.n_sum = S.head == MRL_HEAD_GAUSS ? S.A : 0;
    a.gh = S.A + a.n_sum;
    a.ept = nullptr;
  }
  return a;
}

#ifndef MRL_VJP_BIAS_REG  // 1: bias gradients from per-lane register partials (no per-tile LDS row sums)
#define MRL_VJP_BIAS_REG 1
#endif
#ifndef MRL_VJP_MINW  // minimum waves per SIMD the VJP's registers must allow (build switch)
#define MRL_VJP_MINW 1
#endif
template <bool CACHED, bool WIDE, int SH>
__global__ __launch_bounds__(256, MRL_VJP_MINW) void mlp_vjp_kernel(VjpArgs a_in, const float* __restrict__ img,
                                                       const int32_t* __restrict__ skip) {
  const VjpArgs a = vjp_shape<SH>(a_in);
  constexpr int MT0 = WIDE ? 2 : 1;  // 16-input tiles of gW0
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const MlpDims& d = a.d;
  for (int i = threadIdx.x; i < d.total_size / 4; i += 256)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  float* scrA = lds + d.total_size + wave * SCR_FLOATS;
  float* scrB = scrA + 64 * IMG_PAD;
  const int A = d.A;

  f32x16 gW1[2][2];
  f32x4 gW2[4], gW0[MT0][4];  // 16x16 C tiles: gW2 [unit tile], gW0 [input tile][unit tile]
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) gW1[m][n] = zero16();
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    gW2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MT0; ++m) gW0[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int i16 = lane & 15, kk = lane >> 4;
  float gb0 = 0.f, gb1 = 0.f, gb2 = 0.f;
#if MRL_VJP_BIAS_REG
  // bias gradients as per-lane partials over the wave's tiles (row j of each C tile),
  // summed over the 32 rows once at the end instead of an LDS row sum per tile
  f32x16 pb0[2], pb1[2];
  float pG[4] = {0.f, 0.f, 0.f, 0.f};
  pb0[0] = pb0[1] = pb1[0] = pb1[1] = zero16();
#endif
  float gls[MAX_OUT];
#pragma unroll
  for (int q = 0; q < MAX_OUT; ++q) gls[q] = 0.f;

  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * 4;
  // Every global operand of a tile is issued at the tile's start (h2 and the head rows
  // first, h1 and the gW0 operands, used later, after them).  A register prefetch of
  // the next tile (double buffering) measured slower: its 84 registers went to AGPRs
  // and were copied back every tile (1.11 ms vs 1.00 ms per launch at 4.19 M rows).
  VjpIn<CACHED, WIDE> cur;
  int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  for (; tile < ntiles; tile += stride) {
    vjp_load(a, tile, lane, cur);
    const int64_t row0 = tile * 32;
    Fwd f;
    const float* ct = CACHED ? a.cache + tile * CACHE_TILE_FLOATS : nullptr;
    if constexpr (CACHED) {
#if MRL_VJP_MINW == 1
      // h1 is first used after the gh1 chain: its loads are issued after the ones the
      // first phases wait for
      cache_load(ct, lane, 0, f.h1[0]);
      cache_load(ct, lane, 1, f.h1[1]);
#endif
      f.h2[0] = cur.act[0];
      f.h2[1] = cur.act[1];
    } else {
      forward_tile_pre(lds, d, cur.x0, lane, f);
    }
#if MRL_VJP_MINW == 1
    vjp_load_xg<WIDE>(a, tile, lane, cur.xg);  // used last
#endif

    // head gradient rows in C layout: register r of half h = out r + 4h (masked here,
    // not at load time: see vjp_load)
    const bool valid = row0 + j < a.n;
    float G[4];  // head-gradient rows: register r of half h = output r + 4h
#pragma unroll
    for (int r = 0; r < 4; ++r) G[r] = (valid && r + 4 * h < A) ? cur.g[r] : 0.f;
#if MRL_VJP_BIAS_REG
#pragma unroll
    for (int r = 0; r < 4; ++r) pG[r] += G[r];
#endif
#pragma unroll
    for (int q = 0; q < MAX_OUT; ++q) gls[q] += (valid && h == 0 && q < a.n_sum) ? cur.gs[q] : 0.f;
    // Phase order keeps the MFMA pipe fed: every LDS transpose is issued while an
    // independent MFMA chain runs (the wave_lds barriers split scheduling regions, so
    // the source order is the schedule).  Accumulation orders are unchanged.
    // (a) transposes that need nothing computed: h2 image, G rows
    write_img(scrA, f.h2, lane);
    {
      const int base = (j & 1) * 16 + (j >> 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) scrB[(r + 4 * h) * IMG_PAD + base] = G[r];
    }
    // (b) gh2 = W2 . G   (K = outs, 4 k-steps) while the transposes land
    f32x16 g2[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      g2[mi] = zero16();
      const float4 w = frag4(lds, d.ba2, 4, mi, 0, lane);
      g2[mi] = MFMA32(w.x, G[0], g2[mi]);
      g2[mi] = MFMA32(w.y, G[1], g2[mi]);
      g2[mi] = MFMA32(w.z, G[2], g2[mi]);
      g2[mi] = MFMA32(w.w, G[3], g2[mi]);
    }
    WAVE_LDS_ORDER();
    // (c) gW2 += H2^T G  (row index as K through LDS; 16x16x4, head outputs as N)
    // k-steps 0-3 then 4-7, each half's operands read just before it (the same MFMA
    // order as one pass; half the live operand registers)
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const float4 bq = ld4(scrB + i16 * IMG_PAD + 8 * kk + 4 * hq);
      float4 aq[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) aq[mt] = ld4(scrA + (16 * mt + i16) * IMG_PAD + 8 * kk + 4 * hq);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#ifndef MRL_VJP_ABL_NOGW2
          gW2[mt] = MFMA16(f4get(aq[mt], q), f4get(bq, q), gW2[mt]);
#else
          ;
#endif
#if MRL_VJP_MINW > 1
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
#if !MRL_VJP_BIAS_REG
    if (lane < A) gb2 += rowsum32(scrB, lane);
#endif
    // (d) ga2 = gh2 * (1 - h2^2)
#pragma unroll
    for (int m = 0; m < 2; ++m) mul_dtanh16(g2[m], f.h2[m]);
#if MRL_VJP_BIAS_REG
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) pb1[m][r] += g2[m][r];
#endif
#if MRL_VJP_MINW > 1
    // two waves per SIMD: h1 is loaded once h2 is dead (the other wave covers the
    // latency), keeping the tile's live registers within 256
    if constexpr (CACHED) {
      __builtin_amdgcn_sched_barrier(0);
      cache_load(ct, lane, 0, f.h1[0]);
      cache_load(ct, lane, 1, f.h1[1]);
    }
#endif
    // (e) gh1 = W1 . ga2: registers + the weight image only, so its 64 MFMAs cover the
    //     h1 / ga2 transposes issued next
    f32x16 g1[2];
    g1[0] = zero16();
    g1[1] = zero16();
#ifndef MRL_VJP_ABL_NOCHAIN
#if MRL_VJP_MINW > 1
    // one k-group's weight fragments live at a time (the fence stops the scheduler
    // from hoisting all sixteen ds_read_b128 of the chain)
#pragma unroll
    for (int s4 = 0; s4 < 8; ++s4) {
#pragma unroll
      for (int mo = 0; mo < 2; ++mo) {
        const float4 w = frag4(lds, d.ba1, 32, mo, s4, lane);
        const int s = 4 * s4;
        g1[mo] = MFMA32(w.x, g2[(s + 0) >> 4][(s + 0) & 15], g1[mo]);
        g1[mo] = MFMA32(w.y, g2[(s + 1) >> 4][(s + 1) & 15], g1[mo]);
        g1[mo] = MFMA32(w.z, g2[(s + 2) >> 4][(s + 2) & 15], g1[mo]);
        g1[mo] = MFMA32(w.w, g2[(s + 3) >> 4][(s + 3) & 15], g1[mo]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#else
    chain<2>(lds, d.ba1, g2, lane, g1);
#endif
#endif
    WAVE_LDS_ORDER();
    write_img(scrA, f.h1, lane);
    write_img(scrB, g2, lane);
    WAVE_LDS_ORDER();
#if MRL_VJP_MINW > 1
    vjp_load_xg<WIDE>(a, tile, lane, cur.xg);  // used by (g), under gW1's MFMAs
#endif
    // (f) gW1 += H1^T GA2, and ga1 = gh1 * (1 - h1^2) on the VALU under it
#pragma unroll
    for (int s4 = 0; s4 < VJP_ABL_S4; ++s4) {
      const float4 a0 = ld4(scrA + j * IMG_PAD + h * 16 + 4 * s4);
      const float4 a1 = ld4(scrA + (32 + j) * IMG_PAD + h * 16 + 4 * s4);
      const float4 b0 = ld4(scrB + j * IMG_PAD + h * 16 + 4 * s4);
      const float4 b1 = ld4(scrB + (32 + j) * IMG_PAD + h * 16 + 4 * s4);
      gW1[0][0] = MFMA32(a0.x, b0.x, gW1[0][0]);
      gW1[0][1] = MFMA32(a0.x, b1.x, gW1[0][1]);
      gW1[1][0] = MFMA32(a1.x, b0.x, gW1[1][0]);
      gW1[1][1] = MFMA32(a1.x, b1.x, gW1[1][1]);
      gW1[0][0] = MFMA32(a0.y, b0.y, gW1[0][0]);
      gW1[0][1] = MFMA32(a0.y, b1.y, gW1[0][1]);
      gW1[1][0] = MFMA32(a1.y, b0.y, gW1[1][0]);
      gW1[1][1] = MFMA32(a1.y, b1.y, gW1[1][1]);
      gW1[0][0] = MFMA32(a0.z, b0.z, gW1[0][0]);
      gW1[0][1] = MFMA32(a0.z, b1.z, gW1[0][1]);
      gW1[1][0] = MFMA32(a1.z, b0.z, gW1[1][0]);
      gW1[1][1] = MFMA32(a1.z, b1.z, gW1[1][1]);
      gW1[0][0] = MFMA32(a0.w, b0.w, gW1[0][0]);
      gW1[0][1] = MFMA32(a0.w, b1.w, gW1[0][1]);
      gW1[1][0] = MFMA32(a1.w, b0.w, gW1[1][0]);
      gW1[1][1] = MFMA32(a1.w, b1.w, gW1[1][1]);
#if MRL_VJP_MINW > 1
      __builtin_amdgcn_sched_barrier(0);  // one k-group's operands live at a time
#endif
    }
#if !MRL_VJP_BIAS_REG
    gb1 += rowsum32(scrB, lane);
#endif
#pragma unroll
    for (int m = 0; m < 2; ++m) mul_dtanh16(g1[m], f.h1[m]);
#if MRL_VJP_BIAS_REG
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) pb0[m][r] += g1[m][r];
#endif
    WAVE_LDS_ORDER();
    write_img(scrB, g1, lane);
    WAVE_LDS_ORDER();
    // (g) gW0 += X^T GA1 : A[i = input][k = row] straight from global x (16x16x4)
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      float4 bq[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bq[nt] = ld4(scrB + (16 * nt + i16) * IMG_PAD + 8 * kk + 4 * hq);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int mt = 0; mt < MT0; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
#ifndef MRL_VJP_ABL_NOGW0
            gW0[mt][nt] = MFMA16(cur.xg[8 * mt + 4 * hq + q4], f4get(bq[nt], q4), gW0[mt][nt]);
#else
          ;
#endif
#if MRL_VJP_MINW > 1
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
#if !MRL_VJP_BIAS_REG
    gb0 += rowsum32(scrB, lane);
#endif
    WAVE_LDS_ORDER();
    (void)row0;
  }

  // per-wave partial gradient in flat theta layout
  float* out = a.slab + ((int64_t)blockIdx.x * 4 + wave) * d.P;
#pragma unroll
  for (int mt = 0; mt < MT0; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * mt + 4 * kk + r;
        if (i < d.O) out[d.tW0 + i * HID + 16 * nt + i16] = gW0[mt][nt][r];
      }
#if MRL_VJP_BIAS_REG
  // sum each partial over the 32 rows (lanes j of a half, butterfly), then lane j = 0
  // of half h holds units 32 m + cperm(r, h)
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      pb0[m][r] = half_sum(pb0[m][r]);
      pb1[m][r] = half_sum(pb1[m][r]);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) pG[r] = half_sum(pG[r]);
  if (j == 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        out[d.tb0 + 32 * m + cperm(r, h)] = pb0[m][r];
        out[d.tb1 + 32 * m + cperm(r, h)] = pb1[m][r];
      }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r + 4 * h < A) out[d.tb2 + r + 4 * h] = pG[r];
  }
  (void)gb0;
  (void)gb1;
  (void)gb2;
#else
  out[d.tb0 + lane] = gb0;
#endif
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int mj = 0; mj < 2; ++mj)
#pragma unroll
      for (int r = 0; r < 16; ++r) out[d.tW1 + (32 * mi + cperm(r, h)) * HID + 32 * mj + j] = gW1[mi][mj][r];
#if !MRL_VJP_BIAS_REG
  out[d.tb1 + lane] = gb1;
#endif
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (i16 < A) out[d.tW2 + (16 * mt + 4 * kk + r) * A + i16] = gW2[mt][r];
#if !MRL_VJP_BIAS_REG
  if (lane < A) out[d.tb2 + lane] = gb2;
#endif
  for (int q = 0; q < a.n_sum; ++q) {
    const float s = wave_sumf(gls[q]);
    if (lane == 0) out[d.tls + q] = s;
  }
}

// ------------------------------------------------------------------ cached VJP, 16-row tiles
// The weight gradients sum over rows (K = rows), so their MFMA operands need the row
// index on the lane groups; the backprop chain sums over units, so its operands need
// the unit index there.  The kernel above gets both from one layout through LDS
// transposes.  This one never transposes: on v_mfma_f32_16x16x4_f32 a 16-row tile has
// two register layouts (c = lane & 15, g = lane >> 4, r = register 0..3 of a tile):
//   R  D[unit][row]: lane holds row c, units 16 nt + 4 g + r   (K = units operand)
//   T  D[row][unit]: lane holds unit 16 nt + c, rows 4 g + r   (K = rows operand)
// and every product is issued in the orientation that yields the layout its consumer
// needs: gh2 = W2 G in both (4 MFMAs each: K = head outputs), ga2_R . W1^T gives gh1 in
// T, so ga1 is born in T; the primal activations are read from the cache in the layout
// each use needs (h1 in T, h2 in R and T; the second read of a tile hits L2).
//   gW2 += h2_T^T . G     gW1 += h1_T^T . ga2_T     gW0 += x^T . ga1_T     (K = rows)
//   gh1_T = ga2_R . W1^T                                                   (K = units)
// MFMA work per 16 rows: 4 + 4 + 16 + 64 + 64 + 16 MT0 (168 at O <= 16), the same cycles
// per row as the 32-row kernel minus every LDS transpose; the tile state fits 256
// registers, so a CU runs 8 waves (2 per SIMD) and one wave's loads and VALU work issue
// under the other's MFMAs.  Same sums as the kernel above in a different row / k order
// (fp32 rounding differs, not bitwise equal to it).  The W1 and W2 fragments are read
// straight from the BA1 / BA2 segments of the image (mlp_layout.h).
constexpr int VJP16_WAVES = 8;
// a 0 / 1 factor the optimiser cannot see through: v * opaque(m) stays a multiply, so the
// load of v is not sunk into a branch on m (hipcc drains every outstanding load at such a
// branch's join, the prefetch with it)
__device__ inline float opaque(float m) {
  asm volatile("" : "+v"(m));
  return m;
}
// 16 B per lane global -> LDS (global_load_lds_dwordx4): lane L's bytes land at l + 16 L
// (l wave-uniform); no VGPR destination
template <int AUX = 0>  // AUX: cache-policy bits of the load (2 = nt)
__device__ inline void glds16(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, AUX);
}
constexpr int VJP16_W_FLOATS = 2 * 32 * 64 + 2 * 4 * 64;  // BA1 + BA2 of the image
constexpr int VJP16_H1_FLOATS = 16 * 64;                  // h1 of one 16-row tile
// cache offset (floats) of element (32-row tile's row j, unit w of 32-unit slot `slot`)
__device__ inline int cache_off(int slot, int j, int w) {
  return ((slot * 4 + (w >> 3)) * 64 + 32 * ((w >> 2) & 1) + j) * 4 + (w & 3);
}

// HYB: the two 64x64x16 products of a tile -- gh1_T = ga2_R W1^T and gW1 += h1_T^T ga2_T,
// 128 of its 168 f32 MFMAs -- on v_mfma_f32_16x16x32_bf16 with every f32 operand split
// exactly into three bf16 parts (split2) and the six part products i + j <= 2 kept (each
// dropped one <= 2^-25 |ab|, below one f32 ulp; mlp_split.hip header).  gh1: K = 64 units
// in two k-steps of 32, k = 8 g + e <-> unit 16 (2 s + (e >> 2)) + 4 g + (e & 3), so the A
// fragment is this lane's own ga2_R registers and W1^T comes from a split image built in
// LDS at entry.  gW1: K = the tile's 16 rows, two part products stacked per MFMA (k < 4:
// part P of rows 4 g + k, k >= 4: part Q), three MFMAs for the six products.  MFMA cycles
// per 16-row tile 5,376 -> 2,816; the split costs 48 values of VALU per lane.
template <bool WIDE, bool EPT, bool HYB = false>
__global__ __launch_bounds__(64 * VJP16_WAVES, 2) void mlp_vjp16_kernel(VjpArgs a, const float* __restrict__ img,
                                                                     const int32_t* __restrict__ skip) {
  constexpr int MT0 = WIDE ? 2 : 1;
  // two LDS objects: the LDS-DMA target (h1 staging) apart from the weight fragments, so
  // the compiler's wait for an LDS-DMA in flight is not put in front of fragment reads
  __shared__ __attribute__((aligned(16))) float lds[VJP16_W_FLOATS];
  __shared__ __attribute__((aligned(16))) float sH[VJP16_WAVES * 2 * VJP16_H1_FLOATS];
  // HYB: B fragments of gh1 = ga2 W1^T, [k-step s][tile nt][part p][lane], 24 KB
  __shared__ __attribute__((aligned(16))) bf16x8 wbs[HYB ? 2 * 4 * 3 * 64 : 1];
  if (skip != nullptr && *skip != 0) return;
  const MlpDims& d = a.d;
  // BA1 (W1 fragments, 4096 floats) then BA2 (W2 fragments, 512): contiguous in the image
  for (int i = threadIdx.x; i < VJP16_W_FLOATS / 4; i += 64 * VJP16_WAVES)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img + d.ba1)[i];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile bases
  const int A = d.A, gh = a.gh;
  const int KS2 = (A + 3) >> 2;  // head k-steps (A <= 8)
  // W2 fragment (nt, ks) = W2[16 nt + c][4 ks + g] (zero past A): BA2 holds W2[i][o] at
  // ((i >> 5) * 64 + 32 (o >> 2) + (i & 31)) * 4 + (o & 3)
  const float* w2l = lds + 2 * 32 * 64 + 4 * c + g;
  auto w2frag = [&](int nt, int ks) { return w2l[((nt >> 1) * 64 + 32 * ks + 16 * (nt & 1)) * 4]; };
  __syncthreads();
  // W1 fragment (nt, mt): W1[16 nt + c][16 mt + 4 g + 0..3] as one float4 of BA1
  const float* w1l = lds + (32 * (g & 1) + c) * 4;
  auto w1frag = [&](int nt, int mt) {
    const int s4 = 4 * (mt >> 1) + 2 * (mt & 1) + (g >> 1);
    return ld4(w1l + (((nt >> 1) * 8 + s4) * 64 + 16 * (nt & 1)) * 4);
  };
  // per-lane parts of the cache offsets (cache_off): T gathers (unit 16 p + c, row 4 g + r)
  // and R float4s (row c, units 16 p + 4 g .. + 3); the (slot, p, r) parts are constants
  const int offT = ((c >> 3) * 64 + 32 * ((c >> 2) & 1) + 4 * g) * 4 + (c & 3);
  const int offR = ((g >> 1) * 64 + 32 * (g & 1) + c) * 4;
  if constexpr (HYB) {
    // wave w builds (k-step s = w >> 2, tile nt = w & 3): lane (c, g) element e is
    // W1[16 nt + c][16 (2 s + (e >> 2)) + 4 g + (e & 3)], i.e. w1frag(nt, 2 s + (e >> 2))
    static_assert(VJP16_WAVES == 8, "one (s, nt) per wave");
    const int s = wave >> 2, nt = wave & 3;
    const float4 u = w1frag(nt, 2 * s), v = w1frag(nt, 2 * s + 1);
    bf16x4 pu[3], pv[3];
    split4(f32x4{u.x, u.y, u.z, u.w}, pu);
    split4(f32x4{v.x, v.y, v.z, v.w}, pv);
#pragma unroll
    for (int p = 0; p < 3; ++p) wbs[((s * 4 + nt) * 3 + p) * 64 + lane] = cat4(pu[p], pv[p]);
    __syncthreads();
  }

  f32x4 gW1[4][4], gW2[4], gW0[MT0][4];
  f32x4 zero4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    gW2[m] = zero4;
#pragma unroll
    for (int n = 0; n < 4; ++n) gW1[m][n] = zero4;
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0) gW0[m0][m] = zero4;
  }
  float pb1[4] = {0.f, 0.f, 0.f, 0.f}, pG = 0.f;

  const int64_t ntiles = (a.n + 15) / 16, last = a.n - 1;
  const int64_t stride = (int64_t)gridDim.x * VJP16_WAVES;
  // Tile inputs, loaded one tile ahead (software pipeline at two waves per SIMD): the
  // head-gradient operands and h2 of tile t+1 are issued once tile t's chain has consumed
  // half of ga2_R (its registers are free), h1 and x once the chain is done.  The loads
  // keep raw values; the row / column masks are applied when the tile uses them (a mask
  // at load time would wait for the load there).  Every load is unconditional (clamped
  // addresses) and masked by opaque 0 / 1 factors: a select on a loaded value lets hipcc
  // sink the load into a branch and drain every outstanding load at the join.
  float gq[2], GB[4], xA[MT0][4], xN[MT0][4];  // xN: the next tile's x, moved to xA after gW0
  int32_t et[4], eN[4];
  f32x4 h2R[4], h2T[4], h1T[4];
  // G[row0 + c][4 ks + g] (operand of both gh2 products), G[row0 + 4 g + r][c] (B operand of
  // gW2, bias / logstd sums), h2 in R and T layouts
  auto load_g_h2 = [&](int64_t t) {
    const float* ct = a.cache + (t >> 1) * CACHE_TILE_FLOATS + 16 * (int)(t & 1) * 4;
    const int64_t row0 = t * 16;
    {
      const int64_t rr = row0 + c;
      const float* gr = a.ghead + (rr < last ? rr : last) * gh;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int o = 4 * ks + g;
        gq[ks] = gr[o < gh ? o : gh - 1];
      }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float4 v = ld4(ct + (2 + (nt >> 1)) * 1024 + 512 * (nt & 1) + offR);
      h2R[nt] = f32x4{v.x, v.y, v.z, v.w};
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) h2T[nt][r] = ct[(2 + (nt >> 1)) * 1024 + 512 * (nt & 1) + 4 * r + offT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t rr = row0 + 4 * g + r;
      GB[r] = a.ghead[(rr < last ? rr : last) * gh + (c < gh ? c : gh - 1)];
    }
  };
  auto mask_g = [&](int64_t t) {
    const int64_t row0 = t * 16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) gq[ks] *= opaque((row0 + c < a.n && 4 * ks + g < A && ks < KS2) ? 1.f : 0.f);
#pragma unroll
    for (int r = 0; r < 4; ++r) GB[r] *= opaque((row0 + 4 * g + r < a.n && c < gh) ? 1.f : 0.f);
  };
  // x[row0 + 4 g + r][16 m0 + c] (A operand of gW0; rows past n: any finite value, their
  // ga1 is 0)
  auto take_x = [&]() {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) xA[m0][r] = xN[m0][r];
      if constexpr (EPT) et[r] = eN[r];
    }
  };
  auto load_x = [&](int64_t t) {
    const int64_t row0 = t * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t rr = row0 + 4 * g + r, rc = rr < last ? rr : last;
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) {
        const int col = 16 * m0 + c;
        xN[m0][r] = a.x[rc * a.n_obs + (col < a.n_obs ? col : a.n_obs - 1)];
      }
      if constexpr (EPT) eN[r] = a.ept[rc];
    }
  };
  // h1 of a tile staged in LDS by four LDS-DMA instructions (no registers while in
  // flight).  The 16-B chunks (run = (slot * 4 + q) * 2 + h, row j) of the cache tile land
  // at (run * 16 + jj) * 4 with the rows of each 4-row group rotated by k = 2 (q & 1) + h,
  // jj = 4 (j >> 2) + ((j + k) & 3): the T reads below (lane (c, g): run of unit 16 p + c,
  // row 4 g + r) then hit 64 distinct banks.  The rotation is applied on the source side
  // (an LDS-DMA destination is lane-linear).
  float* const h1s = sH + wave * 2 * VJP16_H1_FLOATS;
  auto dma_h1 = [&](int64_t t, int b) {
    const float* ct = a.cache + (t >> 1) * CACHE_TILE_FLOATS + 16 * (int)(t & 1) * 4;
    const int jj = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int run = 4 * i + (lane >> 4), sq = run >> 1, hh = run & 1, k = 2 * (sq & 1) + hh;
      const int j = 4 * (jj >> 2) + ((jj - k) & 3);
      glds16(ct + (sq * 64 + 32 * hh + j) * 4, h1s + b * VJP16_H1_FLOATS + i * 256);
    }
  };
  // lane parts of the T read offsets: run bits from c, rotated row 4 g + ((r + (c >> 2)) & 3)
  int offH[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    offH[r] = ((c >> 3) * 2 + ((c >> 2) & 1)) * 64 + 16 * g + 4 * ((r + (c >> 2)) & 3) + (c & 3);
  auto read_h1 = [&](int b, int nt) {
    const float* p = h1s + b * VJP16_H1_FLOATS + (nt >> 1) * 512 + (nt & 1) * 256;
    h1T[nt] = f32x4{p[offH[0]], p[offH[1]], p[offH[2]], p[offH[3]]};
  };
  // column O reads 1 (a ones column: gW0's row O is the bias gradient sum_rows ga1); the
  // VF time feature t / timestep_limit at column n_obs as XGlobal computes it
  auto mask_x = [&]() {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) {
        const int col = 16 * m0 + c;
        float xv = xA[m0][r] * opaque(col < a.n_obs ? 1.f : 0.f) + (col == d.O ? 1.f : 0.f);
        if constexpr (EPT) xv += (float)((double)et[r] / a.ts_limit) * opaque(col == a.n_obs ? 1.f : 0.f);
        xA[m0][r] = xv;
      }
  };
  int64_t t = (int64_t)blockIdx.x * VJP16_WAVES + wave;
  if (t < ntiles) {
    load_g_h2(t);
    load_x(t);
    dma_h1(t, 0);
    take_x();
  }
  int buf = 0;
  for (; t < ntiles; t += stride) {
    // the next tile of this wave (the last one re-reads its own tile: loads only)
    const int64_t tn = t + stride < ntiles ? t + stride : t;
    mask_g(t);
    // ---- gh2 in both layouts (K = head outputs), then ga2 = gh2 (1 - h2^2)
    f32x4 ga2R[4], ga2T[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float w = w2frag(nt, 0);
      ga2R[nt] = MFMA16(w, gq[0], zero4);
      ga2T[nt] = MFMA16(gq[0], w, zero4);
    }
    if (KS2 > 1) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float w = w2frag(nt, 1);
        ga2R[nt] = MFMA16(w, gq[1], ga2R[nt]);
        ga2T[nt] = MFMA16(gq[1], w, ga2T[nt]);
      }
    }
    // gW2 += h2_T^T G  (k-step r: rows 4 g + r)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) gW2[nt] = MFMA16(h2T[nt][r], GB[r], gW2[nt]);
#pragma unroll
    for (int r = 0; r < 4; ++r) pG += GB[r];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ga2R[nt][r] *= dtanh(h2R[nt][r]);
        ga2T[nt][r] *= dtanh(h2T[nt][r]);
      }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) pb1[nt] += (ga2T[nt][0] + ga2T[nt][1]) + (ga2T[nt][2] + ga2T[nt][3]);
    __builtin_amdgcn_sched_barrier(0);
    // ---- gh1_T = ga2_R . W1^T (K = units, k-step (mt, r)) interleaved with
    //      gW1 += h1_T^T ga2_T (K = rows): independent chains, one MFMA stream
    f32x4 g1T[4] = {zero4, zero4, zero4, zero4};
    // this tile's h1 (its DMA was issued with the loads phase 1 waited for): all of it is
    // read before the next tile's DMA is issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) read_h1(buf, nt);
    if constexpr (HYB) {
      // gW1 += h1_T^T ga2_T first (ga2_T's registers are free after it): K = 16 rows, two
      // part products per MFMA
      if constexpr (EPT) {  // the VF net's form (the window layout below spills there)
        bf16x4 gp[4][3];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) split4(ga2T[nt], gp[nt]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          bf16x4 hp[3];
          split4(h1T[mt], hp);
          const bf16x8 H21 = cat4(hp[2], hp[1]), H01 = cat4(hp[0], hp[1]), H00 = cat4(hp[0], hp[0]);
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            gW1[mt][nt] = MFMAB16(H21, cat4(gp[nt][0], gp[nt][1]), gW1[mt][nt]);  // h2 g0 + h1 g1
            gW1[mt][nt] = MFMAB16(H01, cat4(gp[nt][2], gp[nt][0]), gW1[mt][nt]);  // h0 g2 + h1 g0
            gW1[mt][nt] = MFMAB16(H00, cat4(gp[nt][1], gp[nt][0]), gW1[mt][nt]);  // h0 g1 + h0 g0
          }
        }
      } else {
        bf16x16 gw[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gw[nt] = split4w(ga2T[nt]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const bf16x16 hw = split4w(h1T[mt]);
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            gW1[mt][nt] = MFMAB16(W8(hw), W0(gw[nt]), gW1[mt][nt]);  // h2 g0 + h0 g1
            gW1[mt][nt] = MFMAB16(W0(hw), W8(gw[nt]), gW1[mt][nt]);  // h0 g2 + h1 g0
            gW1[mt][nt] = MFMAB16(W0(hw), W0(gw[nt]), gW1[mt][nt]);  // h0 g0 + h1 g1
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's G / h2 / x / h1 loads, under the gh1 chain
      load_g_h2(tn);
      load_x(tn);
      dma_h1(tn, buf ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      // gh1_T = ga2_R W1^T: two k-steps of 32 units, six part products each (smallest first)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x4 pa[3], pb[3];
        split4(ga2R[2 * s], pa);
        split4(ga2R[2 * s + 1], pb);
        const bf16x8 A0 = cat4(pa[0], pb[0]), A1 = cat4(pa[1], pb[1]), A2 = cat4(pa[2], pb[2]);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const bf16x8* w = wbs + (s * 4 + nt) * 3 * 64 + lane;
          const bf16x8 B0 = w[0], B1 = w[64], B2 = w[128];
          g1T[nt] = MFMAB16(A2, B0, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B2, g1T[nt]);
          g1T[nt] = MFMAB16(A1, B1, g1T[nt]);
          g1T[nt] = MFMAB16(A1, B0, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B1, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B0, g1T[nt]);
        }
      }
    } else {
    // 16 steps (mt, nt), each W1 fragment read from LDS one step ahead of its MFMAs
    float4 wf = w1frag(0, 0);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int mt = st >> 2, nt = st & 3;
      const float4 wn = st + 1 < 16 ? w1frag((st + 1) & 3, (st + 1) >> 2) : wf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        g1T[nt] = MFMA16(ga2R[mt][r], f4get(wf, r), g1T[nt]);
        gW1[mt][nt] = MFMA16(h1T[mt][r], ga2T[nt][r], gW1[mt][nt]);
      }
      wf = wn;
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's G / h2 loads, once ga2_R of mt 0 and 1 is consumed (its registers
      // are free), under the rest of the chain
      if (st == 7) {
        load_g_h2(tn);
        load_x(tn);
        dma_h1(tn, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    }
    // ---- ga1 = gh1 (1 - h1^2) in T;  gW0 += x^T ga1
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) g1T[nt][r] *= dtanh(h1T[nt][r]);
    mask_x();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gW0[m0][nt] = MFMA16(xA[m0][r], g1T[nt][r], gW0[m0][nt]);
    take_x();
    buf ^= 1;
  }

  // ---- bias / logstd partials: sum over the four lane groups (rows)
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) pb1[nt] = xor32_add(xor16_add(pb1[nt]));
  pG = xor32_add(xor16_add(pG));

  // ---- waves w and w + 4 of the block add their partials through sH (two rounds: gW1,
  // then the rest), waves 0..3 store one slab row each: the slab keeps mrl_slab_rows = 4
  // per block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) h1 DMA has landed
  __syncthreads();  // every wave is done with its h1 buffers
  float* pair = sH + (wave & 3) * 64 * 64;
  if (wave >= 4) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) pair[((m * 4 + n) * 4 + r) * 64 + lane] = gW1[m][n][r];
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) gW1[m][n][r] += pair[((m * 4 + n) * 4 + r) * 64 + lane];
  }
  __syncthreads();
  {
    auto xfer = [&](float v, int k) {
      if (wave >= 4) pair[k * 64 + lane] = v;
    };
    int k = 0;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) xfer(gW2[n][r], k++);
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) xfer(gW0[m0][n][r], k++);
#pragma unroll
    for (int n = 0; n < 4; ++n) xfer(pb1[n], k++);
    xfer(pG, k++);
  }
  __syncthreads();
  if (wave >= 4) return;
  {
    auto pl = [&](int k) { return pair[k * 64 + lane]; };
    int k = 0;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) gW2[n][r] += pl(k++);
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) gW0[m0][n][r] += pl(k++);
#pragma unroll
    for (int n = 0; n < 4; ++n) pb1[n] += pl(k++);
    pG += pl(k++);
  }
  float* out = a.slab + ((int64_t)blockIdx.x * 4 + wave) * d.P;
  // gW1 [in][out]: in = 16 mt + 4 g + r, out = 16 nt + c
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[d.tW1 + (16 * m + 4 * g + r) * HID + 16 * n + c] = gW1[m][n][r];
  // gW2 [u][o]: u = 16 nt + 4 g + r, o = c
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (c < A) out[d.tW2 + (16 * n + 4 * g + r) * A + c] = gW2[n][r];
  // gW0 [i][u]: i = 16 m0 + 4 g + r, u = 16 nt + c; row O (the ones column) is b0's
#pragma unroll
  for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * m0 + 4 * g + r;
        if (i < d.O) out[d.tW0 + i * HID + 16 * n + c] = gW0[m0][n][r];
        else if (i == d.O) out[d.tb0 + 16 * n + c] = gW0[m0][n][r];
      }
  if (g == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) out[d.tb1 + 16 * n + c] = pb1[n];
    if (c < A) out[d.tb2 + c] = pG;
    else if (c < gh) out[d.tls + (c - A)] = pG;
  }
}

// The one-pass Fisher product (mlp_fisher_hyb_kernel): the hybrid VJP above with the
// Fisher product's JVP half beside it in the block.  Waves 0-3 (one per SIMD) run the
// split-operand JVP rows of 32-row tiles (JvpSplitRole, fvp_split_role.h) and leave each
// tile's KL-metric head-gradient rows in an LDS mailbox; waves 4-7 (the partner wave of
// each SIMD) run this VJP on them one round later -- the tile's h1 / h2 / x re-read from
// L2, where the JVP wave's loads of the same CU just put them, so the activation cache
// crosses HBM once per product instead of twice, and each SIMD interleaves the JVP's VALU
// work with the VJP's MFMA chains.  One s_barrier per round (two mailbox slots); the
// head-gradient rows never reach HBM.
constexpr int MBOX_GH = 2 * MAX_OUT;  // mailbox row pitch (floats): the widest head-gradient row
// diagnostic builds only (tools/role_probe.sh): 1 = the VJP role skips its tiles, 2 = the
// JVP role does -- the launch time of the other role alone at the same barriers; 3 = no
// barrier between the rounds (wrong results: the cost of the rounds' lockstep)
#ifndef MRL_FISHER_ROLE_PROBE
#define MRL_FISHER_ROLE_PROBE 0
#endif
// L2 reuse of the activation cache between the roles (round 6): each role alone reads the
// algorithmic 2.33 GB per Hopper product, the pair 4.35 GB -- the VJP role's re-reads of a
// tile a round after the JVP role's miss the XCD's 4 MB L2 (each round brings ~4.5 MB per
// XCD: both roles' reads plus the JVP's prefetch of the next tile; profiles/r06g_fisher_l2.txt).
// MRL_FISHER_JVP_PF 0 (the default): the JVP role loads a tile's x / h1 in the tile's own
// round, not a round ahead -- 4.35 -> 3.98 GB and 1.309 -> 1.277 ms per product;
// MRL_FISHER_VJP_NT 1: the VJP role's loads (the last use of those bytes) non-temporal --
// 3.57 GB (3.34 with both) but 1.32 ms: not kept
#ifndef MRL_FISHER_JVP_PF
#define MRL_FISHER_JVP_PF 0
#endif
#ifndef MRL_FISHER_VJP_NT
#define MRL_FISHER_VJP_NT 0
#endif
// diagnostic builds only: issue priority of one role's waves (s_setprio 1; 1 = the VJP
// role, 2 = the JVP role) -- 0, the default, leaves both at the same priority
#ifndef MRL_FISHER_PRIO
#define MRL_FISHER_PRIO 0
#endif
__device__ inline f32x4 ldv4(const f32x4* p) {
  if constexpr (MRL_FISHER_VJP_NT) return __builtin_nontemporal_load(p);
  return *p;
}
__device__ inline float ldv1(const float* p) {
  if constexpr (MRL_FISHER_VJP_NT) return __builtin_nontemporal_load(p);
  return *p;
}

struct FisherFusedIn {
  RowsArgs ra;        // the producer rows' arguments (x, n, inv_ng, logstd / dlogstd, cache;
                      // PROD 1: act / adv / oldprob / partial, the cache written)
  BDims rb;
  const float* img_s; // split images of theta and of the tangent (mrl_mlp_pack_split)
  const float* imt_s; // (PROD 1: unused)
};

// PROD: what waves 0-3 produce for the VJP role.  0: the Fisher product's JVP rows (the KL
// metric's head-gradient rows along a tangent, reading the activation cache); 1: the
// policy gradient's forward rows (round 6, mrl_mlp_grad_hyb) -- the SURRGRAD pass of
// mlp_rows_split_kernel (split_rows_tile, the same per-row code), which writes the
// activation cache the VJP role then reads and the surrogate head-gradient rows into the
// mailbox, and leaves the surr / KL / entropy sums per producer wave in the partial rows
template <int SH, int PROD = 0>
__global__ __launch_bounds__(64 * VJP16_WAVES, 1) void mlp_fisher_hyb_kernel(VjpArgs a, const float* __restrict__ img,
                                                                           const int32_t* __restrict__ skip,
                                                                           FisherFusedIn fz) {
  constexpr int MT0 = 1;
  // LDS: the W2 fragments (the split W1^T of gh1 is in wbs), h1 staging of the four VJP
  // waves, wbs, the mailbox and (dynamic) the two split images: 148 KB for Hopper
  __shared__ __attribute__((aligned(16))) float lds[2 * 4 * 64];
  __shared__ __attribute__((aligned(16))) float sH[4 * 2 * VJP16_H1_FLOATS];
  // B fragments of gh1 = ga2 W1^T, [k-step s][tile nt][part p][lane], 24 KB
  __shared__ __attribute__((aligned(16))) bf16x8 wbs[2 * 4 * 3 * 64];
  // head-gradient rows of the JVP waves' tiles, [slot][JVP wave][row][MBOX_GH]
  // PROD 1 runs the VJP two rounds behind (LAG): its prefetch of the next tile then reads
  // cache rows the producer finished a round earlier; NSLOT mailbox slots per JVP wave
  constexpr int LAG = PROD == 1 ? 2 : 1, NSLOT = LAG + 1;
  __shared__ __attribute__((aligned(16))) float mbox[NSLOT * 4 * 32 * MBOX_GH];
  extern __shared__ __attribute__((aligned(16))) float ldsx[];  // the two split images
  if (skip != nullptr && *skip != 0) return;
  const MlpDims& d = a.d;
  for (int i = threadIdx.x; i < 2 * 4 * 64 / 4; i += 64 * VJP16_WAVES)  // BA2 of the image
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img + d.ba1 + 2 * 32 * 64)[i];
  const int WS = split_fwd_words(fz.rb);
  for (int i = threadIdx.x; i < WS / 4; i += 64 * VJP16_WAVES) {
    reinterpret_cast<float4*>(ldsx)[i] = reinterpret_cast<const float4*>(fz.img_s)[i];
    if constexpr (PROD == 0) reinterpret_cast<float4*>(ldsx + WS)[i] = reinterpret_cast<const float4*>(fz.imt_s)[i];
  }
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile bases
  const int A = d.A, gh = a.gh;
  const int KS2 = (A + 3) >> 2;  // head k-steps (A <= 8)
  // W2 fragment (nt, ks) = W2[16 nt + c][4 ks + g] (zero past A): BA2 holds W2[i][o] at
  // ((i >> 5) * 64 + 32 (o >> 2) + (i & 31)) * 4 + (o & 3)
  const float* w2l = lds + 4 * c + g;
  auto w2frag = [&](int nt, int ks) { return w2l[((nt >> 1) * 64 + 32 * ks + 16 * (nt & 1)) * 4]; };
  __syncthreads();
  // W1 fragment (nt, mt): W1[16 nt + c][16 mt + 4 g + 0..3] as one float4 of BA1 (read
  // from the image in global memory, only to build wbs)
  const float* w1l = img + d.ba1 + (32 * (g & 1) + c) * 4;
  auto w1frag = [&](int nt, int mt) {
    const int s4 = 4 * (mt >> 1) + 2 * (mt & 1) + (g >> 1);
    return ld4(w1l + (((nt >> 1) * 8 + s4) * 64 + 16 * (nt & 1)) * 4);
  };
  // per-lane parts of the cache offsets (cache_off): T gathers (unit 16 p + c, row 4 g + r)
  // and R float4s (row c, units 16 p + 4 g .. + 3); the (slot, p, r) parts are constants
  const int offT = ((c >> 3) * 64 + 32 * ((c >> 2) & 1) + 4 * g) * 4 + (c & 3);
  const int offR = ((g >> 1) * 64 + 32 * (g & 1) + c) * 4;
  {
    // wave w builds (k-step s = w >> 2, tile nt = w & 3): lane (c, g) element e is
    // W1[16 nt + c][16 (2 s + (e >> 2)) + 4 g + (e & 3)], i.e. w1frag(nt, 2 s + (e >> 2))
    static_assert(VJP16_WAVES == 8, "one (s, nt) per wave");
    const int s = wave >> 2, nt = wave & 3;
    const float4 u = w1frag(nt, 2 * s), v = w1frag(nt, 2 * s + 1);
    bf16x4 pu[3], pv[3];
    split4(f32x4{u.x, u.y, u.z, u.w}, pu);
    split4(f32x4{v.x, v.y, v.z, v.w}, pv);
#pragma unroll
    for (int p = 0; p < 3; ++p) wbs[((s * 4 + nt) * 3 + p) * 64 + lane] = cat4(pu[p], pv[p]);
    __syncthreads();
  }
  // Rounds: in round r the JVP waves fill mailbox slot r & 1 with the rows of their
  // round-r tiles (32-row tile T = (r G + block) 4 + w) and the VJP waves consume slot
  // (r - 1) & 1; every wave passes the same number of barriers (one per round)
  const int64_t nt32 = (a.n + 31) / 32, stride32 = (int64_t)gridDim.x * 4;
  const int64_t rounds = (nt32 + stride32 - 1) / stride32 + LAG;
  auto fused_barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's mailbox writes / reads are done
    if (MRL_FISHER_ROLE_PROBE != 3) __builtin_amdgcn_s_barrier();  // 3: timing build without the rounds' barrier
    asm volatile("" ::: "memory");
  };
  if constexpr (PROD == 1) {
    if (wave < 4) {
      RowsArgs ra = fz.ra;
      BDims rb = fz.rb;
      split_shape<SH>(ra, rb);
      const MlpDims dd = head_dims(ra.d, rb);
      float ls[MAX_OUT], sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
      for (int j = 0; j < MAX_OUT; ++j) {
        ls[j] = (ra.logstd != nullptr && j < ra.A) ? ra.logstd[j] : 0.f;
        sd[j] = expf(ls[j]);
        dls[j] = 0.f;
      }
      const int A = ra.A, actw = ra.head == MRL_HEAD_SOFTMAX ? 1 : A, opw = ra.head == MRL_HEAD_SOFTMAX ? A : 2 * A;
      double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
      int64_t T = (int64_t)blockIdx.x * 4 + wave;
      for (int64_t r = 0; r < rounds; ++r) {
        if (r + LAG < rounds && T < nt32) {
          // the row epilogue's inputs at this tile's rows and its head-gradient row in the
          // mailbox (pitch MBOX_GH; rows past n get zeros, as the JVP role's)
          float* mb = mbox + ((r % NSLOT) * 4 + wave) * 32 * MBOX_GH;
          const int64_t row0 = T * 32;
          RowsArgs ae = ra;
          ae.adv = ra.adv + row0;
          ae.act = ra.head == MRL_HEAD_SOFTMAX ? (const void*)(reinterpret_cast<const int32_t*>(ra.act) + row0)
                                               : (const void*)(reinterpret_cast<const float*>(ra.act) + row0 * actw);
          ae.oldprob = ra.oldprob + row0 * opw;
          ae.ghead = mb;
          ae.gh = MBOX_GH;
          if ((lane >> 5) == 0 && row0 + (lane & 31) >= ra.n)
            for (int j = 0; j < MBOX_GH; ++j) mb[(lane & 31) * MBOX_GH + j] = 0.f;
          split_rows_tile<MRL_EPI_SURRGRAD, true>(ra, rb, ldsx, dd, lane, T, true, ls, sd, dls, acc0, acc1, acc2, ae,
                                            lane & 31);
          T += stride32;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's cache rows are in L2 for the VJP waves
        fused_barrier();
      }
      acc0 = wave_sum(acc0);
      acc1 = wave_sum(acc1);
      acc2 = wave_sum(acc2);
      if (lane == 0) {
        double* p = ra.partial + ((int64_t)blockIdx.x * 4 + wave) * 4;
        p[0] = acc0;
        p[1] = acc1;
        p[2] = acc2;
        p[3] = 0.0;
      }
      return;
    }
  } else {
    if (wave < 4) {
      RowsArgs ra = fz.ra;
      BDims rb = fz.rb;
      split_shape<SH>(ra, rb);
      JvpSplitRole role;
      role.init(ra, rb, ldsx, ldsx + WS, lane);
      if constexpr (MRL_FISHER_PRIO == 2) __builtin_amdgcn_s_setprio(1);
      float sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
      for (int j = 0; j < MAX_OUT; ++j) {
        sd[j] = expf((ra.logstd != nullptr && j < ra.A) ? ra.logstd[j] : 0.f);
        dls[j] = (ra.dlogstd != nullptr && j < ra.A) ? ra.dlogstd[j] : 0.f;
      }
      int64_t T = (int64_t)blockIdx.x * 4 + wave;
      if (MRL_FISHER_JVP_PF && T < nt32) role.prologue(T);
      for (int64_t r = 0; r < rounds; ++r) {
        if (MRL_FISHER_ROLE_PROBE != 2 && r + 1 < rounds && T < nt32) {
          const int64_t tn = T + stride32 < nt32 ? T + stride32 : T;  // the last tile re-reads itself
          float* mb = mbox + ((r & 1) * 4 + wave) * 32 * MBOX_GH + (lane & 31) * MBOX_GH;
          role.template tile<MRL_FISHER_JVP_PF != 0>(T, tn, [&](bool valid, int64_t, const float (&z)[MAX_OUT],
                                                                  const float (&dz)[MAX_OUT]) {
            if ((lane >> 5) == 0) {
              // the KL-metric head-gradient row (row_epilogue FVP); rows past n hold 0
              float gg[MAX_OUT], gl[MAX_OUT];
              fvp_metric_row<MAX_OUT>(ra, z, dz, sd, dls, gg, gl);
#pragma unroll
              for (int j = 0; j < MAX_OUT; ++j)
                if (j < ra.A) {
                  mb[j] = valid ? gg[j] : 0.f;
                  if (ra.head == MRL_HEAD_GAUSS) mb[ra.A + j] = valid ? gl[j] : 0.f;
                }
            }
          });
          T += stride32;
        }
        fused_barrier();
      }
      return;
    }
  }

  if constexpr (MRL_FISHER_PRIO == 1 && PROD == 0) __builtin_amdgcn_s_setprio(1);
  f32x4 gW1[4][4], gW2[4], gW0[MT0][4];
  f32x4 zero4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    gW2[m] = zero4;
#pragma unroll
    for (int n = 0; n < 4; ++n) gW1[m][n] = zero4;
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0) gW0[m0][m] = zero4;
  }
  float pb1[4] = {0.f, 0.f, 0.f, 0.f}, pG = 0.f;

  const int64_t last = a.n - 1;
  // Tile inputs, loaded one tile ahead (software pipeline at two waves per SIMD): the
  // head-gradient operands and h2 of tile t+1 are issued once tile t's chain has consumed
  // half of ga2_R (its registers are free), h1 and x once the chain is done.  The loads
  // keep raw values; the row / column masks are applied when the tile uses them (a mask
  // at load time would wait for the load there).  Every load is unconditional (clamped
  // addresses) and masked by opaque 0 / 1 factors: a select on a loaded value lets hipcc
  // sink the load into a branch and drain every outstanding load at the join.
  float gq[2], GB[4], xA[MT0][4], xN[MT0][4];  // xN: the next tile's x, moved to xA after gW0
  f32x4 h2R[4], h2T[4], h1T[4];
  // h2 in R and T layouts
  auto load_h2 = [&](int64_t t) {
    const float* ct = a.cache + (t >> 1) * CACHE_TILE_FLOATS + 16 * (int)(t & 1) * 4;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      h2R[nt] = ldv4(reinterpret_cast<const f32x4*>(ct + (2 + (nt >> 1)) * 1024 + 512 * (nt & 1) + offR));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) h2T[nt][r] = ldv1(ct + (2 + (nt >> 1)) * 1024 + 512 * (nt & 1) + 4 * r + offT);
  };
  // G of 16-row tile t from its 32-row tile's mailbox rows mbt: G[row0 + c][4 ks + g]
  // (operand of both gh2 products), G[row0 + 4 g + r][c] (B operand of gW2, bias / logstd sums)
  const float* mbt = mbox;
  auto load_g_mbox = [&](int64_t t) {
    const float* m = mbt + 16 * (int)(t & 1) * MBOX_GH;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int o = 4 * ks + g;
      gq[ks] = m[c * MBOX_GH + (o < gh ? o : gh - 1)];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) GB[r] = m[(4 * g + r) * MBOX_GH + (c < gh ? c : gh - 1)];
  };
  auto mask_g = [&](int64_t t) {
    const int64_t row0 = t * 16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) gq[ks] *= opaque((row0 + c < a.n && 4 * ks + g < A && ks < KS2) ? 1.f : 0.f);
#pragma unroll
    for (int r = 0; r < 4; ++r) GB[r] *= opaque((row0 + 4 * g + r < a.n && c < gh) ? 1.f : 0.f);
  };
  // x[row0 + 4 g + r][16 m0 + c] (A operand of gW0; rows past n: any finite value, their
  // ga1 is 0)
  auto take_x = [&]() {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) xA[m0][r] = xN[m0][r];
    }
  };
  auto load_x = [&](int64_t t) {
    const int64_t row0 = t * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t rr = row0 + 4 * g + r, rc = rr < last ? rr : last;
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) {
        const int col = 16 * m0 + c;
        xN[m0][r] = ldv1(a.x + rc * a.n_obs + (col < a.n_obs ? col : a.n_obs - 1));
      }
    }
  };
  // h1 of a tile staged in LDS by four LDS-DMA instructions (no registers while in
  // flight).  The 16-B chunks (run = (slot * 4 + q) * 2 + h, row j) of the cache tile land
  // at (run * 16 + jj) * 4 with the rows of each 4-row group rotated by k = 2 (q & 1) + h,
  // jj = 4 (j >> 2) + ((j + k) & 3): the T reads below (lane (c, g): run of unit 16 p + c,
  // row 4 g + r) then hit 64 distinct banks.  The rotation is applied on the source side
  // (an LDS-DMA destination is lane-linear).
  float* const h1s = sH + (wave - 4) * 2 * VJP16_H1_FLOATS;
  auto dma_h1 = [&](int64_t t, int b) {
    const float* ct = a.cache + (t >> 1) * CACHE_TILE_FLOATS + 16 * (int)(t & 1) * 4;
    const int jj = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int run = 4 * i + (lane >> 4), sq = run >> 1, hh = run & 1, k = 2 * (sq & 1) + hh;
      const int j = 4 * (jj >> 2) + ((jj - k) & 3);
      glds16<MRL_FISHER_VJP_NT ? 2 : 0>(ct + (sq * 64 + 32 * hh + j) * 4, h1s + b * VJP16_H1_FLOATS + i * 256);
    }
  };
  // lane parts of the T read offsets: run bits from c, rotated row 4 g + ((r + (c >> 2)) & 3)
  int offH[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    offH[r] = ((c >> 3) * 2 + ((c >> 2) & 1)) * 64 + 16 * g + 4 * ((r + (c >> 2)) & 3) + (c & 3);
  auto read_h1 = [&](int b, int nt) {
    const float* p = h1s + b * VJP16_H1_FLOATS + (nt >> 1) * 512 + (nt & 1) * 256;
    h1T[nt] = f32x4{p[offH[0]], p[offH[1]], p[offH[2]], p[offH[3]]};
  };
  // column O reads 1 (a ones column: gW0's row O is the bias gradient sum_rows ga1)
  auto mask_x = [&]() {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0) {
        const int col = 16 * m0 + c;
        float xv = xA[m0][r] * opaque(col < a.n_obs ? 1.f : 0.f) + (col == d.O ? 1.f : 0.f);
        xA[m0][r] = xv;
      }
  };
  int buf = 0;
  // one 16-row tile t, the loads of tile tn issued under its chain
  auto vjp_tile = [&](int64_t t, int64_t tn) {
    load_g_mbox(t);
    mask_g(t);
    // ---- gh2 in both layouts (K = head outputs), then ga2 = gh2 (1 - h2^2)
    f32x4 ga2R[4], ga2T[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float w = w2frag(nt, 0);
      ga2R[nt] = MFMA16(w, gq[0], zero4);
      ga2T[nt] = MFMA16(gq[0], w, zero4);
    }
    if (KS2 > 1) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float w = w2frag(nt, 1);
        ga2R[nt] = MFMA16(w, gq[1], ga2R[nt]);
        ga2T[nt] = MFMA16(gq[1], w, ga2T[nt]);
      }
    }
    // gW2 += h2_T^T G  (k-step r: rows 4 g + r)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) gW2[nt] = MFMA16(h2T[nt][r], GB[r], gW2[nt]);
#pragma unroll
    for (int r = 0; r < 4; ++r) pG += GB[r];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ga2R[nt][r] *= dtanh(h2R[nt][r]);
        ga2T[nt][r] *= dtanh(h2T[nt][r]);
      }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) pb1[nt] += (ga2T[nt][0] + ga2T[nt][1]) + (ga2T[nt][2] + ga2T[nt][3]);
    __builtin_amdgcn_sched_barrier(0);
    // ---- gh1_T = ga2_R . W1^T (K = units, k-step (mt, r)) interleaved with
    //      gW1 += h1_T^T ga2_T (K = rows): independent chains, one MFMA stream
    f32x4 g1T[4] = {zero4, zero4, zero4, zero4};
    // this tile's h1 (its DMA was issued with the loads phase 1 waited for): all of it is
    // read before the next tile's DMA is issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) read_h1(buf, nt);
    {
      // gW1 += h1_T^T ga2_T first (ga2_T's registers are free after it): K = 16 rows, two
      // part products per MFMA
      {
        bf16x16 gw[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gw[nt] = split4w(ga2T[nt]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const bf16x16 hw = split4w(h1T[mt]);
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            gW1[mt][nt] = MFMAB16(W8(hw), W0(gw[nt]), gW1[mt][nt]);  // h2 g0 + h0 g1
            gW1[mt][nt] = MFMAB16(W0(hw), W8(gw[nt]), gW1[mt][nt]);  // h0 g2 + h1 g0
            gW1[mt][nt] = MFMAB16(W0(hw), W0(gw[nt]), gW1[mt][nt]);  // h0 g0 + h1 g1
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's h2 / x / h1 loads, under the gh1 chain
      load_h2(tn);
      load_x(tn);
      dma_h1(tn, buf ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      // gh1_T = ga2_R W1^T: two k-steps of 32 units, six part products each (smallest first)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x4 pa[3], pb[3];
        split4(ga2R[2 * s], pa);
        split4(ga2R[2 * s + 1], pb);
        const bf16x8 A0 = cat4(pa[0], pb[0]), A1 = cat4(pa[1], pb[1]), A2 = cat4(pa[2], pb[2]);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const bf16x8* w = wbs + (s * 4 + nt) * 3 * 64 + lane;
          const bf16x8 B0 = w[0], B1 = w[64], B2 = w[128];
          g1T[nt] = MFMAB16(A2, B0, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B2, g1T[nt]);
          g1T[nt] = MFMAB16(A1, B1, g1T[nt]);
          g1T[nt] = MFMAB16(A1, B0, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B1, g1T[nt]);
          g1T[nt] = MFMAB16(A0, B0, g1T[nt]);
        }
      }
    }
    // ---- ga1 = gh1 (1 - h1^2) in T;  gW0 += x^T ga1
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) g1T[nt][r] *= dtanh(h1T[nt][r]);
    mask_x();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gW0[m0][nt] = MFMA16(xA[m0][r], g1T[nt][r], gW0[m0][nt]);
    take_x();
    buf ^= 1;
  };
  {
    const int vw = wave - 4;
    int64_t T = (int64_t)blockIdx.x * 4 + vw;
    // the first tile's inputs: before round 0's barrier (PROD 0: the cache is read-only
    // here), or after it (PROD 1: the producer wrote them in round 0)
    for (int64_t r = 0; r < LAG; ++r) {
      if (r == LAG - 1 && T < nt32) {
        load_h2(2 * T);
        load_x(2 * T);
        dma_h1(2 * T, 0);
        take_x();
      }
      fused_barrier();  // round r: the producer waves fill slot r
    }
    for (int64_t r = LAG; r < rounds; ++r) {
      if (MRL_FISHER_ROLE_PROBE != 1 && T < nt32) {
        mbt = mbox + (((r - LAG) % NSLOT) * 4 + vw) * 32 * MBOX_GH;
        const int64_t Tn = T + stride32 < nt32 ? T + stride32 : T;  // the last tile re-reads itself
#pragma unroll 1
        for (int hf = 0; hf < 2; ++hf) vjp_tile(2 * T + hf, hf ? 2 * Tn : 2 * T + 1);
        T += stride32;
      }
      fused_barrier();
    }
  }

  // ---- bias / logstd partials: sum over the four lane groups (rows)
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) pb1[nt] = xor32_add(xor16_add(pb1[nt]));
  pG = xor32_add(xor16_add(pG));

  // ---- the four VJP waves store one slab row each (mrl_slab_rows = 4 per block)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) h1 DMA has landed
  float* out = a.slab + ((int64_t)blockIdx.x * 4 + (wave - 4)) * d.P;
  // gW1 [in][out]: in = 16 mt + 4 g + r, out = 16 nt + c
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[d.tW1 + (16 * m + 4 * g + r) * HID + 16 * n + c] = gW1[m][n][r];
  // gW2 [u][o]: u = 16 nt + 4 g + r, o = c
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (c < A) out[d.tW2 + (16 * n + 4 * g + r) * A + c] = gW2[n][r];
  // gW0 [i][u]: i = 16 m0 + 4 g + r, u = 16 nt + c; row O (the ones column) is b0's
#pragma unroll
  for (int m0 = 0; m0 < MT0; ++m0)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * m0 + 4 * g + r;
        if (i < d.O) out[d.tW0 + i * HID + 16 * n + c] = gW0[m0][n][r];
        else if (i == d.O) out[d.tb0 + 16 * n + c] = gW0[m0][n][r];
      }
  if (g == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) out[d.tb1 + 16 * n + c] = pb1[n];
    if (c < A) out[d.tb2 + c] = pG;
    else if (c < gh) out[d.tls + (c - A)] = pG;
  }
}

// ------------------------------------------------------------------ pack / reduce
__global__ void mlp_pack_kernel(MlpDims d, const float* __restrict__ th, float* __restrict__ image, int count,
                                const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) image[i] = image_value(d, th, i);
}

// RG row groups of 64 columns per block (blockDim = 64 * RG); group g sums rows
// g, g + RG, ... with 8 independent accumulators (8 loads in flight per lane), then
// the RG group sums are added in a fixed pairwise order
template <class T, class O, int RG = 4>
__global__ void reduce_rows_kernel(const T* __restrict__ slab, int64_t rows, int64_t cols, O* __restrict__ out,
                                   const int32_t* __restrict__ skip) {
  __shared__ double part[RG][64];
  if (skip != nullptr && *skip != 0) return;
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + c;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < cols) {
    int64_t r = g;
    for (; r + 7 * RG < rows; r += 8 * RG) {
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += (double)slab[(r + RG * q) * cols + col];
    }
    for (; r < rows; r += RG) s[0] += (double)slab[r * cols + col];
  }
  part[g][c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if constexpr (RG == 4) {
    if (g == 0 && col < cols) out[col] = (O)(((part[0][c] + part[1][c]) + part[2][c]) + part[3][c]);
  } else {
#pragma unroll
    for (int w = RG / 2; w >= 1; w >>= 1) {
      if (g < w) part[g][c] += part[g + w][c];
      __syncthreads();
    }
    if (g == 0 && col < cols) out[col] = (O)part[0][c];
  }
}

// few columns (per-wave loss partials): one block per column, 256 threads over rows
template <class T, class O>
__global__ void reduce_rows_narrow_kernel(const T* __restrict__ slab, int64_t rows, int64_t cols, O* __restrict__ out,
                                          const int32_t* __restrict__ skip) {
  __shared__ double red[256];
  if (skip != nullptr && *skip != 0) return;
  const int64_t col = blockIdx.x;
  double s = 0.0;
  for (int64_t r = threadIdx.x; r < rows; r += 256) s += (double)slab[r * cols + col];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[col] = (O)red[0];
}

// per-row probtype values on probability rows (mrl_probtype_rows): the helpers the
// row epilogues use, one thread per row
__global__ void probtype_rows_kernel(int head, int A, int64_t n, const float* __restrict__ prob,
                                     const float* __restrict__ prob2, const void* __restrict__ x,
                                     float* __restrict__ loglik, float* __restrict__ kl, float* __restrict__ ent) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (head == MRL_HEAD_SOFTMAX) {
      const float* p = prob + r * A;
      if (loglik) loglik[r] = logf(p[reinterpret_cast<const int32_t*>(x)[r]]);
      if (kl) {
        const float* q = prob2 + r * A;
        float k = 0.f;
        for (int j = 0; j < A; ++j) k += cat_kl_term(p[j], q[j]);
        kl[r] = k;
      }
      if (ent) {
        float h = 0.f;
        for (int j = 0; j < A; ++j) h += cat_ent_term(p[j]);
        ent[r] = h;
      }
    } else {
      const float* p = prob + r * 2 * A;
      float sumlog = 0.f;
      for (int j = 0; j < A; ++j) sumlog += logf(p[A + j]);
      if (loglik) {
        const float* xv = reinterpret_cast<const float*>(x) + r * A;
        float q = 0.f;
        for (int j = 0; j < A; ++j) {
          const float u = (xv[j] - p[j]) / p[A + j];
          q += u * u;
        }
        loglik[r] = gauss_loglik(q, sumlog, A);
      }
      if (kl) {
        const float* p2 = prob2 + r * 2 * A;
        float k = 0.f;
        for (int j = 0; j < A; ++j) k += gauss_kl_term(p[j], p[A + j], p2[j], p2[A + j]);
        kl[r] = k - 0.5f * A;
      }
      if (ent) ent[r] = gauss_entropy(sumlog, A);
    }
  }
}

}  // namespace mrl

using namespace mrl;

static int check_desc(const mrl_mlp_desc* d) {
  if (d == nullptr) return fail(E_ARG, "null mlp desc");
  if (d->n_hidden != HID || d->n_layers != 2)
    return fail(E_UNSUPPORTED, "only hid_sizes=[64,64] is implemented on the HIP path (got " +
                                   std::to_string(d->n_layers) + "x" + std::to_string(d->n_hidden) + ")");
  if (d->n_in < 1 || d->n_in > MAX_IN) return fail(E_UNSUPPORTED, "n_in must be in [1, 32]");
  if (d->n_out < 1 || d->n_out > MAX_OUT) return fail(E_UNSUPPORTED, "n_out must be in [1, 8]");
  if (d->head < 0 || d->head > 2) return fail(E_ARG, "bad head kind");
  if (d->head == MRL_HEAD_LINEAR && d->n_out != 1) return fail(E_ARG, "linear head needs n_out=1");
  if (d->cus < 0 || d->cus > 1024) return fail(E_ARG, "cus must be in [0, 1024]");
  return OK;
}

static MlpDims dims_of(const mrl_mlp_desc* d) { return mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS); }

// the static shape (mlp_layout.h) a launch matches, or 0: plain rows only (a time
// feature column built from ep_t takes the generic kernels, except the value nets'
// prediction pass: time_ok, SH_TIME variants)
static int static_shape_of(const mrl_mlp_desc* d, bool has_ept, bool time_ok = false) {
#ifdef MRL_NO_STATIC_SHAPES
  (void)d;
  (void)has_ept;
  (void)time_ok;
  return 0;
#else
  if (has_ept && !time_ok) return 0;
  for (int i = 1; i < N_STATIC_SHAPES; ++i)
    if (STATIC_SHAPES[i].O == d->n_in && STATIC_SHAPES[i].A == d->n_out && STATIC_SHAPES[i].head == d->head) {
      if (!has_ept) return i;
      return STATIC_SHAPES[i].head == MRL_HEAD_LINEAR ? (i | SH_TIME) : 0;
    }
  return 0;
#endif
}

// grid caps for passes sized for `cus` CUs (the caps are per 256): the VJP runs one
// block per CU, so on a fit stream of 192 CUs a 256-block grid would take two rounds
static int64_t desc_cus(const mrl_mlp_desc* d) { return d != nullptr && d->cus > 0 ? d->cus : 256; }
static int64_t rows_blocks(int64_t n, int64_t cus = 256) {
  int64_t b = ceil_div(ceil_div(n, 32), 4);
  if (b < 1) b = 1;
  const int64_t cap = ROWS_MAX_BLOCKS * cus / 256 > 0 ? ROWS_MAX_BLOCKS * cus / 256 : 1;
  return b > cap ? cap : b;
}
static int64_t vjp_blocks(int64_t n, int64_t cus = 256) {
  int64_t b = ceil_div(ceil_div(n, 32), 4);
  if (b < 1) b = 1;
  const int64_t cap = VJP_MAX_BLOCKS * cus / 256 > 0 ? VJP_MAX_BLOCKS * cus / 256 : 1;
  return b > cap ? cap : b;
}

extern "C" {

const char* mrl_last_error(void) { return mrl::g_err.c_str(); }
int32_t mrl_version(void) { return 1; }

int64_t mrl_mlp_num_params(const mrl_mlp_desc* d) {
  if (check_desc(d) != OK) return -1;
  return dims_of(d).P;
}
int64_t mrl_mlp_image_floats(const mrl_mlp_desc* d) {
  if (check_desc(d) != OK) return -1;
  return dims_of(d).total_size;
}
int64_t mrl_partial_rows(int64_t n) { return rows_blocks(n) * 4; }
int64_t mrl_act_cache_floats(int64_t n) { return ceil_div(n, 32) * CACHE_TILE_FLOATS; }
int64_t mrl_slab_rows(int64_t n) { return vjp_blocks(n) * 4; }
// 1 when the one-pass Fisher product applies to the net's shape: a policy MLP of a static
// shape (Hopper-v2, CartPole-v0) whose input fits the 16-row VJP (O % 16 != 0, O <= 16)
// and whose two split images fit one block's LDS beside the VJP's (W2 fragments, h1
// staging, split W1^T, mailbox)
int32_t mrl_mlp_fisher_hyb_fits(const mrl_mlp_desc* d) {
  if (d == nullptr || d->n_hidden != HID || d->n_layers != 2 || d->head == MRL_HEAD_LINEAR) return 0;
  if (d->n_out < 1 || d->n_out > MAX_OUT || d->n_in < 1 || d->n_in > MAX_IN) return 0;
  const MlpDims m = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  if (m.O > 16 || m.O % 16 == 0) return 0;
  // the static shapes only (the run-time-shape instantiation spills at 256 registers)
  if (static_shape_of(d, false) == 0) return 0;
  const size_t lds = (size_t)split_fwd_words(bf16_dims(d->n_in, d->n_out)) * 4 * 2 + 2 * 4 * 64 * 4 +
                     4 * 2 * VJP16_H1_FLOATS * 4 + 2 * 4 * 3 * 64 * 16 + 2 * 4 * 32 * MBOX_GH * 4;
  return lds <= 160 * 1024 ? 1 : 0;
}
int64_t mrl_mlp_partial_rows(const mrl_mlp_desc* d, int64_t n) {
  if (check_desc(d) != OK) return -1;
  return rows_blocks(n, desc_cus(d)) * 4;
}
int64_t mrl_mlp_slab_rows(const mrl_mlp_desc* d, int64_t n) {
  if (check_desc(d) != OK) return -1;
  return vjp_blocks(n, desc_cus(d)) * 4;
}

int mrl_mlp_pack(const mrl_mlp_desc* d, const float* theta, float* image, int32_t fwd_only, const int32_t* skip,
                 void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!theta || !image) return fail(E_ARG, "null pointer");
  MlpDims m = dims_of(d);
  int count = fwd_only ? m.fwd_size : m.total_size;
  hipLaunchKernelGGL(mlp_pack_kernel, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, m, theta, image,
                     count, skip);
  return hip_check(hipGetLastError(), "mrl_mlp_pack");
}

// the RowsArgs of one row pass and the argument checks of its epilogue (mrl_mlp_rows,
// mrl_mlp_rows_split); 1 = nothing to do (n <= 0)
static int rows_args(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image, const float* tangent,
                     const float* image_t, const mrl_rows_io* io, RowsArgs& a) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!io || !image || !io->x) return fail(E_ARG, "null pointer");
  if (io->n <= 0) return 1;
  a.d = dims_of(d);
  a.head = d->head;
  a.n_obs = d->n_in - (io->ep_t ? 1 : 0);
  a.gh = d->head == MRL_HEAD_GAUSS ? 2 * d->n_out : d->n_out;
  a.A = d->n_out;
  a.x = io->x;
  a.ept = io->ep_t;
  a.ts_limit = io->timestep_limit;
  a.n = io->n;
  a.inv_ng = io->inv_n_global;
  a.act = io->act;
  a.adv = io->adv;
  a.oldprob = io->oldprob;
  a.target = io->target;
  a.out = io->out;
  a.ghead = io->ghead;
  a.partial = io->partial;
  a.logstd = (d->head == MRL_HEAD_GAUSS && theta) ? theta + a.d.tls : nullptr;
  a.dlogstd = (d->head == MRL_HEAD_GAUSS && tangent) ? tangent + a.d.tls : nullptr;
  a.kl_coeff = (float)io->kl_coeff;
  a.kl_cutoff = (float)io->kl_cutoff;
  a.cutoff_coeff = (float)io->cutoff_coeff;
  a.reverse_kl = io->reverse_kl;
  a.cache = io->act_cache;
  a.cache_mode = io->act_cache != nullptr ? io->cache_mode : 0;
  a.feat = io->feat_out;
  if (a.feat != nullptr && (epi != MRL_EPI_PROB || io->ep_t == nullptr))
    return fail(E_ARG, "feat_out is for MRL_EPI_PROB with ep_t (the value prediction)");
  if (a.cache_mode == MRL_CACHE_READ && epi != MRL_EPI_FVP) return fail(E_ARG, "MRL_CACHE_READ is for MRL_EPI_FVP");
  if (a.cache_mode == MRL_CACHE_WRITE && (epi == MRL_EPI_FVP || epi == MRL_EPI_PPOSGD))
    return fail(E_ARG, "MRL_CACHE_WRITE is for the plain forward epilogues");
  switch (epi) {
    case MRL_EPI_PROB:
      if (!io->out) return fail(E_ARG, "EPI_PROB needs out");
      if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
      break;
    case MRL_EPI_LOSSES:
    case MRL_EPI_SURRGRAD:
    case MRL_EPI_PPOGRAD:
    case MRL_EPI_PPOSGD:
      if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "policy epilogue on a value net");
      if (!io->act || !io->adv || !io->oldprob || !io->partial) return fail(E_ARG, "losses need act/adv/oldprob/partial");
      if (epi != MRL_EPI_LOSSES && !io->ghead) return fail(E_ARG, "gradient epilogues need ghead");
      if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
      if (epi == MRL_EPI_PPOSGD && io->n > MRL_PPO_BLOCK_ROWS) return fail(E_ARG, "PPOSGD minibatch exceeds one block");
      break;
    case MRL_EPI_VFLOSS:
      if (d->head != MRL_HEAD_LINEAR || !io->target || !io->ghead || !io->partial)
        return fail(E_ARG, "VFLOSS needs a linear head, target, ghead, partial");
      break;
    case MRL_EPI_FVP:
      if (!tangent || !image_t || !io->ghead) return fail(E_ARG, "FVP needs tangent, image_t, ghead");
      if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
      break;
    default:
      return fail(E_ARG, "unknown epilogue");
  }
  return OK;
}

int mrl_mlp_rows(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image, const float* tangent,
                 const float* image_t, const mrl_rows_io* io, const int32_t* skip, void* stream) {
  RowsArgs a;
  int rc = rows_args(d, epi, theta, image, tangent, image_t, io, a);
  if (rc) return rc > 0 ? OK : rc;
  // cus sizes the passes whose sums follow the grid (per-wave partials); the others
  // (forward / PROB / FVP rows) keep the device-wide grid wherever they run
  const int64_t blocks = rows_blocks(io->n, io->partial != nullptr ? desc_cus(d) : 256);
  size_t shm = (size_t)a.d.fwd_size * 4 * (epi == MRL_EPI_FVP ? 2 : 1);
  hipStream_t s = (hipStream_t)stream;
  const int sh = static_shape_of(d, io->ep_t != nullptr, epi == MRL_EPI_PROB);
  const bool pol = sh == 1 || sh == 2, vf = sh == 3 || sh == 4;
  const dim3 grid(epi == MRL_EPI_PPOSGD ? 1 : blocks), blk(ROWS_BLOCK);
#define MRL_ROWS_LAUNCH(EK, OK)                                                                                     \
  do {                                                                                                              \
    if ((OK) && sh == 1) hipLaunchKernelGGL((mlp_rows_kernel<EK, 1>), grid, blk, shm, s, a, image, image_t, skip); \
    else if ((OK) && sh == 2) hipLaunchKernelGGL((mlp_rows_kernel<EK, 2>), grid, blk, shm, s, a, image, image_t, skip); \
    else if ((OK) && sh == 3) hipLaunchKernelGGL((mlp_rows_kernel<EK, 3>), grid, blk, shm, s, a, image, image_t, skip); \
    else if ((OK) && sh == 4) hipLaunchKernelGGL((mlp_rows_kernel<EK, 4>), grid, blk, shm, s, a, image, image_t, skip); \
    else hipLaunchKernelGGL((mlp_rows_kernel<EK, 0>), grid, blk, shm, s, a, image, image_t, skip);                  \
  } while (0)
  switch (epi) {
    case MRL_EPI_PROB:
      if (sh == (3 | SH_TIME)) hipLaunchKernelGGL((mlp_rows_kernel<MRL_EPI_PROB, 3 | SH_TIME>), grid, blk, shm, s, a, image, image_t, skip);
      else if (sh == (4 | SH_TIME)) hipLaunchKernelGGL((mlp_rows_kernel<MRL_EPI_PROB, 4 | SH_TIME>), grid, blk, shm, s, a, image, image_t, skip);
      else MRL_ROWS_LAUNCH(MRL_EPI_PROB, true);
      break;
    case MRL_EPI_LOSSES: MRL_ROWS_LAUNCH(MRL_EPI_LOSSES, pol); break;
    case MRL_EPI_SURRGRAD: MRL_ROWS_LAUNCH(MRL_EPI_SURRGRAD, pol); break;
    case MRL_EPI_VFLOSS: MRL_ROWS_LAUNCH(MRL_EPI_VFLOSS, vf); break;
    case MRL_EPI_FVP:
      if (a.cache_mode == MRL_CACHE_READ) MRL_ROWS_LAUNCH(EPI_FVP_CACHED, pol);
      else MRL_ROWS_LAUNCH(MRL_EPI_FVP, pol);
      break;
    case MRL_EPI_PPOGRAD: MRL_ROWS_LAUNCH(MRL_EPI_PPOGRAD, pol); break;
    case MRL_EPI_PPOSGD: MRL_ROWS_LAUNCH(MRL_EPI_PPOSGD, pol); break;
  }
#undef MRL_ROWS_LAUNCH
  return hip_check(hipGetLastError(), "mrl_mlp_rows");
}

int mrl_mlp_rows_split(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image_s,
                       const mrl_rows_io* io, const int32_t* skip, void* stream) {
  if (epi != MRL_EPI_PROB && epi != MRL_EPI_LOSSES && epi != MRL_EPI_SURRGRAD && epi != MRL_EPI_VFLOSS)
    return fail(E_UNSUPPORTED, "mrl_mlp_rows_split: PROB, LOSSES, SURRGRAD or VFLOSS");
  if (d != nullptr && (d->n_in > MAX_IN || d->n_out > MAX_OUT || d->n_hidden != HID || d->n_layers != 2))
    return fail(E_UNSUPPORTED, "mrl_mlp_rows_split: the 64-wide fused shape only");
  RowsArgs a;
  int rc = rows_args(d, epi, theta, image_s, nullptr, nullptr, io, a);
  if (rc) return rc > 0 ? OK : rc;
  // the grid (and so the partial rows) of mrl_mlp_rows: mrl_mlp_partial_rows holds for both
  const int64_t blocks = rows_blocks(io->n, io->partial != nullptr ? desc_cus(d) : 256);
  const int sh = static_shape_of(d, io->ep_t != nullptr, epi == MRL_EPI_PROB);
  return launch_rows_split(epi, sh, a, bf16_dims(d->n_in, d->n_out), image_s, blocks, skip, stream);
}

int mrl_mlp_vjp(const mrl_mlp_desc* d, const float* image, const float* x, const int32_t* ep_t, double ts_limit,
                const float* ghead, int64_t n, float* slab, const float* act_cache, const int32_t* skip,
                void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!image || !x || !ghead || !slab) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  VjpArgs a;
  a.d = dims_of(d);
  a.n_obs = d->n_in - (ep_t ? 1 : 0);
  a.n_sum = d->head == MRL_HEAD_GAUSS ? d->n_out : 0;
  a.gh = d->n_out + a.n_sum;
  a.x = x;
  a.ept = ep_t;
  a.ts_limit = ts_limit;
  a.n = n;
  a.ghead = ghead;
  a.slab = slab;
  const int64_t blocks = vjp_blocks(n, desc_cus(d));
  size_t shm = ((size_t)a.d.total_size + 4 * (size_t)SCR_FLOATS) * 4;
  a.cache = act_cache;
  const bool wide = a.d.O > 16;
  // the run-time-shape VJP measured faster than its static-shape instantiations (Hopper
  // policy at 4.19 M rows: 1.02 vs 1.07 ms; the register allocation differs), so the
  // static shapes are used by the rows kernels only
  const int sh = MRL_VJP_MINW > 1 ? static_shape_of(d, ep_t != nullptr) : 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(blocks), blk(256);
#define MRL_VJP_LAUNCH(C)                                                                                   \
  do {                                                                                                      \
    if (sh == 1) hipLaunchKernelGGL((mlp_vjp_kernel<C, false, 1>), grid, blk, shm, s, a, image, skip);     \
    else if (sh == 2) hipLaunchKernelGGL((mlp_vjp_kernel<C, false, 2>), grid, blk, shm, s, a, image, skip); \
    else if (sh == 3) hipLaunchKernelGGL((mlp_vjp_kernel<C, false, 3>), grid, blk, shm, s, a, image, skip); \
    else if (sh == 4) hipLaunchKernelGGL((mlp_vjp_kernel<C, false, 4>), grid, blk, shm, s, a, image, skip); \
    else if (!wide) hipLaunchKernelGGL((mlp_vjp_kernel<C, false, 0>), grid, blk, shm, s, a, image, skip);   \
    else hipLaunchKernelGGL((mlp_vjp_kernel<C, true, 0>), grid, blk, shm, s, a, image, skip);               \
  } while (0)
  // the 16-row kernel takes the bias gradient b0 through a ones column of gW0's padding
  if (act_cache != nullptr && a.d.O % 16 != 0) {
    // the transpose-free 16-row kernel (8 waves per block, same slab rows per block)
    const size_t shm16 = 0;  // static LDS: weight fragments + h1 staging (82 KB)
    const dim3 blk16(64 * VJP16_WAVES);
    const bool ept = ep_t != nullptr;
    if (wide) {
      if (ept) hipLaunchKernelGGL((mlp_vjp16_kernel<true, true>), grid, blk16, shm16, s, a, image, skip);
      else hipLaunchKernelGGL((mlp_vjp16_kernel<true, false>), grid, blk16, shm16, s, a, image, skip);
    } else {
      if (ept) hipLaunchKernelGGL((mlp_vjp16_kernel<false, true, true>), grid, blk16, shm16, s, a, image, skip);
      else hipLaunchKernelGGL((mlp_vjp16_kernel<false, false, true>), grid, blk16, shm16, s, a, image, skip);
    }
    return hip_check(hipGetLastError(), "mrl_mlp_vjp");
  }
  if (act_cache != nullptr) MRL_VJP_LAUNCH(true);
  else MRL_VJP_LAUNCH(false);
#undef MRL_VJP_LAUNCH
  return hip_check(hipGetLastError(), "mrl_mlp_vjp");
}

int mrl_mlp_fisher_hyb(const mrl_mlp_desc* d, const float* theta, const float* image, const float* image_s,
                       const float* tangent, const float* image_t_s, const mrl_rows_io* io, float* slab,
                       const int32_t* skip, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!io || !image || !image_s || !image_t_s || !tangent || !io->x || !slab) return fail(E_ARG, "null pointer");
  if (!io->act_cache || io->cache_mode != MRL_CACHE_READ)
    return fail(E_ARG, "mrl_mlp_fisher_hyb reads the f32 activation cache (MRL_CACHE_READ)");
  if (io->ep_t) return fail(E_ARG, "mrl_mlp_fisher_hyb: policy rows only (no time feature)");
  if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "Fisher product of a value net");
  if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
  if (mrl_mlp_fisher_hyb_fits(d) != 1) return fail(E_UNSUPPORTED, "mrl_mlp_fisher_hyb: shape does not fit one block's LDS");
  if (io->n <= 0) return OK;
  VjpArgs a;
  a.d = dims_of(d);
  a.n_obs = d->n_in;
  a.n_sum = d->head == MRL_HEAD_GAUSS ? d->n_out : 0;
  a.gh = d->n_out + a.n_sum;
  a.x = io->x;
  a.ept = nullptr;
  a.ts_limit = 1.0;
  a.n = io->n;
  a.ghead = nullptr;
  a.slab = slab;
  a.cache = io->act_cache;
  FisherFusedIn fz{};
  RowsArgs& r = fz.ra;
  r.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  r.head = d->head;
  r.n_obs = d->n_in;
  r.gh = a.gh;
  r.A = d->n_out;
  r.x = io->x;
  r.n = io->n;
  r.inv_ng = io->inv_n_global;
  r.logstd = d->head == MRL_HEAD_GAUSS ? theta + r.d.tls : nullptr;
  r.dlogstd = d->head == MRL_HEAD_GAUSS ? tangent + r.d.tls : nullptr;
  r.cache = io->act_cache;
  r.cache_mode = MRL_CACHE_READ;
  fz.rb = bf16_dims(d->n_in, d->n_out);
  fz.img_s = image_s;
  fz.imt_s = image_t_s;
  // the VJP's grid and slab rows (mrl_mlp_slab_rows): one slab row per VJP wave
  const dim3 grid(vjp_blocks(io->n, desc_cus(d))), blk(64 * VJP16_WAVES);
  const size_t shm = (size_t)split_fwd_words(fz.rb) * 4 * 2;
  hipStream_t s = (hipStream_t)stream;
  switch (static_shape_of(d, false)) {
    case 1: hipLaunchKernelGGL((mlp_fisher_hyb_kernel<1>), grid, blk, shm, s, a, image, skip, fz); break;
    default: hipLaunchKernelGGL((mlp_fisher_hyb_kernel<2>), grid, blk, shm, s, a, image, skip, fz); break;
  }
  return hip_check(hipGetLastError(), "mrl_mlp_fisher_hyb");
}

int mrl_mlp_grad_hyb(const mrl_mlp_desc* d, const float* theta, const float* image, const float* image_s,
                     const mrl_rows_io* io, float* slab, const int32_t* skip, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!io || !image || !image_s || !io->x || !slab) return fail(E_ARG, "null pointer");
  if (!io->act || !io->adv || !io->oldprob || !io->partial) return fail(E_ARG, "mrl_mlp_grad_hyb needs act/adv/oldprob/partial");
  if (!io->act_cache || io->cache_mode != MRL_CACHE_WRITE)
    return fail(E_ARG, "mrl_mlp_grad_hyb writes the f32 activation cache (MRL_CACHE_WRITE)");
  if (io->ep_t) return fail(E_ARG, "mrl_mlp_grad_hyb: policy rows only (no time feature)");
  if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "policy gradient of a value net");
  if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
  if (mrl_mlp_fisher_hyb_fits(d) != 1) return fail(E_UNSUPPORTED, "mrl_mlp_grad_hyb: shape does not fit one block's LDS");
  if (io->n <= 0) return OK;
  VjpArgs a;
  a.d = dims_of(d);
  a.n_obs = d->n_in;
  a.n_sum = d->head == MRL_HEAD_GAUSS ? d->n_out : 0;
  a.gh = d->n_out + a.n_sum;
  a.x = io->x;
  a.ept = nullptr;
  a.ts_limit = 1.0;
  a.n = io->n;
  a.ghead = nullptr;
  a.slab = slab;
  a.cache = io->act_cache;
  FisherFusedIn fz{};
  RowsArgs& r = fz.ra;
  r.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  r.head = d->head;
  r.n_obs = d->n_in;
  r.gh = a.gh;
  r.A = d->n_out;
  r.x = io->x;
  r.n = io->n;
  r.inv_ng = io->inv_n_global;
  r.act = io->act;
  r.adv = io->adv;
  r.oldprob = io->oldprob;
  r.partial = io->partial;
  r.logstd = d->head == MRL_HEAD_GAUSS ? theta + r.d.tls : nullptr;
  r.cache = io->act_cache;
  r.cache_mode = MRL_CACHE_WRITE;
  fz.rb = bf16_dims(d->n_in, d->n_out);
  fz.img_s = image_s;
  fz.imt_s = nullptr;
  // the VJP's grid and slab rows (mrl_mlp_slab_rows): one slab row per VJP wave, and one
  // partial row (surr, kl, ent, 0) per producer wave -- the same count
  const dim3 grid(vjp_blocks(io->n, desc_cus(d))), blk(64 * VJP16_WAVES);
  const size_t shm = (size_t)split_fwd_words(fz.rb) * 4;
  hipStream_t s = (hipStream_t)stream;
  switch (static_shape_of(d, false)) {
    case 1: hipLaunchKernelGGL((mlp_fisher_hyb_kernel<1, 1>), grid, blk, shm, s, a, image, skip, fz); break;
    default: hipLaunchKernelGGL((mlp_fisher_hyb_kernel<2, 1>), grid, blk, shm, s, a, image, skip, fz); break;
  }
  return hip_check(hipGetLastError(), "mrl_mlp_grad_hyb");
}

int mrl_probtype_rows(int32_t head, int32_t k, int64_t n, const float* prob, const float* prob2, const void* x,
                      float* loglik, float* kl, float* ent, void* stream) {
  if (head != MRL_HEAD_SOFTMAX && head != MRL_HEAD_GAUSS) return fail(E_ARG, "mrl_probtype_rows: bad head kind");
  if (k < 1) return fail(E_ARG, "mrl_probtype_rows: k < 1");
  if (!prob || (loglik && !x) || (kl && !prob2)) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(probtype_rows_kernel, dim3(std::min<int64_t>(ceil_div(n, 256), 2048)), dim3(256), 0, (hipStream_t)stream, (int)head, (int)k, n,
                     prob, prob2, x, loglik, kl, ent);
  return hip_check(hipGetLastError(), "mrl_probtype_rows");
}

int mrl_reduce_rows_f32(const float* slab, int64_t rows, int64_t cols, float* out, const int32_t* skip, void* stream) {
  if (!slab || !out) return fail(E_ARG, "null pointer");
  if (cols <= 0) return OK;
  // tall slabs (the fused VJP's per-wave rows: 1,024 x 5,126 for Hopper, only 81
  // column blocks wide): 16 row groups (1,024 threads) so the row split fills the chip;
  // short wide ones (the layered GEMMs' split-K slabs, 64 rows) keep 4 groups
  if (rows >= 256)
    hipLaunchKernelGGL((reduce_rows_kernel<float, float, 16>), dim3(ceil_div(cols, 64)), dim3(1024), 0,
                       (hipStream_t)stream, slab, rows, cols, out, skip);
  else
    hipLaunchKernelGGL((reduce_rows_kernel<float, float, 4>), dim3(ceil_div(cols, 64)), dim3(256), 0,
                       (hipStream_t)stream, slab, rows, cols, out, skip);
  return hip_check(hipGetLastError(), "mrl_reduce_rows_f32");
}
int mrl_reduce_rows_f64(const double* slab, int64_t rows, int64_t cols, double* out, const int32_t* skip,
                        void* stream) {
  if (!slab || !out) return fail(E_ARG, "null pointer");
  if (cols <= 0) return OK;
  if (cols <= 16)
    hipLaunchKernelGGL((reduce_rows_narrow_kernel<double, double>), dim3(cols), dim3(256), 0, (hipStream_t)stream,
                       slab, rows, cols, out, skip);
  else
    hipLaunchKernelGGL((reduce_rows_kernel<double, double>), dim3(ceil_div(cols, 64)), dim3(256), 0,
                       (hipStream_t)stream, slab, rows, cols, out, skip);
  return hip_check(hipGetLastError(), "mrl_reduce_rows_f64");
}

// K line-search candidates of the fused policy scored in one call, read back once by the
// caller (trpo.py:143-159): candidates -> per candidate its forward image + a LOSSES pass
// into its own partial rows -> out[k] = the candidate's (surr, kl, ent, n) sums.
int mrl_linesearch_eval(const mrl_mlp_desc* pol, int32_t compute, const float* theta_old, const double* fullstep,
                        int32_t k0, int32_t K, const mrl_rows_io* io, float* cand, float* images, int64_t image_stride,
                        double* partials, int64_t partial_stride, double* out, void* stream) {
  int rc = check_desc(pol);
  if (rc) return rc;
  if (!io || !cand || !images || !partials || !out) return fail(E_ARG, "mrl_linesearch_eval: null pointer");
  if (compute != MRL_COMPUTE_F32 && compute != MRL_COMPUTE_BF16 && compute != MRL_COMPUTE_SPLIT)
    return fail(E_ARG, "bad compute");
  const bool bf = compute == MRL_COMPUTE_BF16, sp = compute == MRL_COMPUTE_SPLIT;
  const int64_t P = mrl_mlp_num_params(pol);
  const int64_t img = bf ? mrl_mlp_image_words_bf16(pol) : sp ? mrl_mlp_image_words_split(pol) : mrl_mlp_image_floats(pol);
  // the LOSSES pass sizes its grid (and so its partial rows) by the desc's CU count
  const int64_t prow = bf ? mrl_mlp_partial_rows_bf16(pol, io->n) : mrl_mlp_partial_rows(pol, io->n);
  if (image_stride < img || partial_stride < prow * 4) return fail(E_ARG, "mrl_linesearch_eval: strides too small");
  rc = mrl_linesearch_candidates(theta_old, fullstep, k0, K, P, cand, stream);
  for (int32_t k = 0; k < K && rc == OK; ++k) {
    const float* th = cand + (int64_t)k * P;
    float* im = images + (int64_t)k * image_stride;
    mrl_rows_io iok = *io;
    iok.partial = partials + (int64_t)k * partial_stride;
    iok.cache_mode = MRL_CACHE_NONE;
    iok.act_cache = nullptr;
    rc = bf ? mrl_mlp_pack_bf16(pol, th, im, 1, nullptr, stream)
            : sp ? mrl_mlp_pack_split(pol, th, im, nullptr, stream) : mrl_mlp_pack(pol, th, im, 1, nullptr, stream);
    if (rc == OK)
      rc = bf ? mrl_mlp_rows_bf16(pol, MRL_EPI_LOSSES, th, im, nullptr, nullptr, &iok, nullptr, stream)
            : sp ? mrl_mlp_rows_split(pol, MRL_EPI_LOSSES, th, im, &iok, nullptr, stream)
                 : mrl_mlp_rows(pol, MRL_EPI_LOSSES, th, im, nullptr, nullptr, &iok, nullptr, stream);
    if (rc == OK) rc = mrl_reduce_rows_f64(iok.partial, prow, 4, out + 4 * (int64_t)k, nullptr, stream);
  }
  return rc;
}

}  // extern "C"
