// bf16 throughput mode of the fused 64-wide MLP kernels (MRL_COMPUTE_BF16): the same
// passes as mlp_kernels.hip (forward + row epilogues, Fisher-product JVP, VJP) on
// v_mfma_f32_32x32x16_bf16 -- 16x the f32 MFMA rate -- with f32 accumulation.
//
// Rounding points (bf16 RNE): the weights W0, W1 (and the tangent's dW0, dW1), the
// layer inputs x, h1, h2 and the backpropagated head rows / layer-2 gradients that
// enter an MFMA.  Biases, tanh, tanh', the head layer (n_out <= 8, f32 VALU on the
// bf16-rounded h2) and every row epilogue stay f32.  fp32 (mlp_kernels.hip) is the
// parity dtype; this mode is checked against the fp64 oracle at a bf16 bound
// (tests/test_gpu_bf16.py).
//
// Layouts.  A 32-row tile keeps activations transposed in the accumulators exactly as
// the f32 kernels do ("F layout", D[unit][row]: row on the lane, 16 units in the
// registers, unit = 32*mt + cperm(r, h)); the C/D layout of the bf16 MFMA is the f32
// one.  Registers 8s'..8s'+7 of a tile, converted to bf16, are the B fragment of a
// k-step whose k index j of lane half h is unit cperm(8s' + j, h): layers chain with
// no data movement, the weight fragments of the image are permuted to match.
// The weight gradients sum over rows (the lane index of an F tile), so the VJP turns
// F tiles into "T layout" tiles D[row][unit] (unit on the lane, rows in the
// registers) with an identity MFMA (X^T . I: exact, the values are bf16 already) and
// feeds T tiles as both operands of X^T . Y -- no LDS transposes at all.
//
// Replaces the same reference functions as mlp_kernels.hip (core.py:269-270,
// trpo.py:68-70, core.py:608, 670-671) in reduced precision.
#include <math.h>
#include <stdlib.h>

#include "../../include/mrl_hip.h"
#include "mlp_device.h"
#include "rows_epilogue.h"
#include "bf16_frag.h"

namespace mrl {

__global__ void mlp_pack_bf16_kernel(MlpDims d, BDims b, const float* __restrict__ th, float* __restrict__ image,
                                     int words, const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  if (w < b.fa0) {
    // f32 section: the f32 image's element at the same segment-relative position
    int idx;
    if (w < b.fb1) idx = d.fb0 + (w - b.fb0);
    else if (w < b.hv) idx = d.fb1 + (w - b.fb1);
    else if (w < b.hb) idx = d.hv + (w - b.hv);
    else idx = d.hb + (w - b.hb);
    image[w] = image_value(d, th, idx);
    return;
  }
  int seg, rel;
  if (w < b.fa1) { seg = 0; rel = w - b.fa0; }
  else if (w < b.bw2) { seg = 1; rel = w - b.fa1; }
  else if (w < b.bt1) { seg = 2; rel = w - b.bw2; }
  else { seg = 3; rel = w - b.bt1; }
  const int frag = rel >> 2, q = rel & 3;
  const __bf16 lo = (__bf16)bimage_elem(d, b, th, seg, frag, 2 * q);
  const __bf16 hi = (__bf16)bimage_elem(d, b, th, seg, frag, 2 * q + 1);
  const uint32_t v = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
  image[w] = __uint_as_float(v);
}

// ---- primal activation cache, bf16: per 32-row tile [layer 2][s 4][lane 64] x 16 B
// (8 KB per tile): every wave load / store instruction moves 1 KB contiguous.
constexpr int BCACHE_TILE_WORDS = 2 * 4 * 64 * 4;
__device__ inline void bcache_store(float* tile, int layer, int lane, const bf16x8* fr) {
#pragma unroll
  for (int s = 0; s < 4; ++s) reinterpret_cast<bf16x8*>(tile)[(layer * 4 + s) * 64 + lane] = fr[s];
}
__device__ inline void bcache_load(const float* tile, int layer, int lane, bf16x8* fr) {
#pragma unroll
  for (int s = 0; s < 4; ++s) fr[s] = reinterpret_cast<const bf16x8*>(tile)[(layer * 4 + s) * 64 + lane];
}

// head partials from a 32-unit tile of bf16-valued h2 (f32 VALU, the f32 kernels' head)
// forward: h1 / h2 fragments (bf16) and, with the f32 head, z
template <class XL>
__device__ inline void forward_b(const float* img, const MlpDims& d, const BDims& b, const XL& xl, int lane,
                                 bf16x8* h1b, bf16x8* h2b, float* z) {
  const int h = lane >> 5;
  bf16x8 xb[MAX_KS0B];
#pragma unroll
  for (int s0 = 0; s0 < MAX_KS0B; ++s0) xb[s0] = s0 < b.KS0B ? x_frag(xl, s0, h) : bf16x8{};
  f32x16 a1[2];
  a1[0] = load_bias16(img, b.fb0, 0, h);
  a1[1] = load_bias16(img, b.fb0, 1, h);
  layer0_b(img, b, xb, lane, a1);
  tanh16(a1[0]);
  tanh16(a1[1]);
#pragma unroll
  for (int s = 0; s < 4; ++s) h1b[s] = pack8(a1[s >> 1], s & 1);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) z[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    f32x16 a = load_bias16(img, b.fb1, mo, h);
    chain_b(img, b, mo, h1b, lane, a);
    __builtin_amdgcn_sched_barrier(0);
    tanh16(a);
    h2b[2 * mo] = pack8(a, 0);
    h2b[2 * mo + 1] = pack8(a, 1);
    const f32x16 ar = unpack16(h2b, mo);
    head_partial_mt(img, d, ar, mo, h, z);  // d = head_dims(...)
    // scheduling fences keep the head's weight reads and the next tile's fragment
    // prefetch from all being hoisted (the static-shape builds otherwise spill)
    __builtin_amdgcn_sched_barrier(0);
  }
  head_finish(img, d, z);
}

// JVP to the head from cached bf16 h1 / h2 fragments (need_z: also the primal head)
template <class XL>
__device__ inline void jvp_b(const float* img, const float* imt, const MlpDims& d, const BDims& b, const XL& xl,
                             int lane, const bf16x8* h1b, const bf16x8* h2b, float* z, float* dz, bool need_z) {
  const int h = lane >> 5;
  bf16x8 xb[MAX_KS0B];
#pragma unroll
  for (int s0 = 0; s0 < MAX_KS0B; ++s0) xb[s0] = s0 < b.KS0B ? x_frag(xl, s0, h) : bf16x8{};
  f32x16 dh[2];
  dh[0] = load_bias16(imt, b.fb0, 0, h);
  dh[1] = load_bias16(imt, b.fb0, 1, h);
  layer0_b(imt, b, xb, lane, dh);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const f32x16 h1 = unpack16(h1b, m);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[m][r] *= dtanh(h1[r]);
  }
  bf16x8 dhb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) dhb[s] = pack8(dh[s >> 1], s & 1);
  float dzt[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    if (need_z) z[o] = 0.f;
    dz[o] = 0.f;
    dzt[o] = 0.f;
  }
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    f32x16 da = load_bias16(imt, b.fb1, mo, h);
    chain_b(img, b, mo, dhb, lane, da);
    chain_b(imt, b, mo, h1b, lane, da);
    const f32x16 a = unpack16(h2b, mo);
#pragma unroll
    for (int r = 0; r < 16; ++r) da[r] *= dtanh(a[r]);
    if (need_z) head_partial_mt(img, d, a, mo, h, z);
    head_partial_mt(img, d, da, mo, h, dz);
    head_partial_mt(imt, d, a, mo, h, dzt);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (need_z) head_finish(img, d, z);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) dz[o] += dzt[o];
  head_finish(imt, d, dz);
}

constexpr int ROWS_BLOCK_B = 256;
constexpr int ROWS_MAX_BLOCKS_B = 3072;
constexpr int EPI_FVP_CACHED_B = 100;

// the kernel arguments with a static shape's dimensions substituted (SH == 0: run time;
// SH | SH_TIME keeps ep_t for the time-feature column)
template <int SH>
__device__ inline void rows_shape_b(RowsArgs& a, BDims& b) {
  if constexpr ((SH & ~SH_TIME) != 0) {
    constexpr int B = SH & ~SH_TIME;
    constexpr StaticShape S = STATIC_SHAPES[B];
    a.d = static_dims(B);
    a.A = S.A;
    a.head = S.head;
    a.n_obs = (SH & SH_TIME) ? S.O - 1 : S.O;
    a.gh = S.head == MRL_HEAD_GAUSS ? 2 * S.A : S.A;
    if constexpr (!(SH & SH_TIME)) a.ept = nullptr;
    b = bf16_dims(S.O, S.A);
  }
}

// waves per SIMD the row kernels are compiled for: 3 (168 VGPRs) for the cached FVP pass
// of the static shapes -- it waits on memory for half its wave time and a third wave
// hides some of it (CartPole 0.313 -> 0.265 ms, Hopper 0.353 -> 0.286 ms at 4.19 M
// rows; Hopper's spills 16 bytes a lane) -- 2 for the others (the loss / gradient passes
// measured level or slower at 3; the run-time shape and the uncached FVP pass spill)
#ifndef MRL_ROWS_B_OCC3
#define MRL_ROWS_B_OCC3 1
#endif
// MRL_ROWS_B_OCC4=1: the PROB / LOSSES / SURRGRAD passes of the static shapes at 4 waves
// (48-64 bytes a lane spilled).  Measured and not kept (tools/occ4_ab.sh): SURRGRAD
// 0.47 -> 0.50 ms (CartPole), 0.52 -> 0.58 ms (Hopper); PROB level
#ifndef MRL_ROWS_B_OCC4
#define MRL_ROWS_B_OCC4 0
#endif
template <int EPI_K, int SH>
constexpr int rows_b_occ() {
  if (MRL_ROWS_B_OCC4 && (SH & ~SH_TIME) != 0 && EPI_K <= MRL_EPI_SURRGRAD) return 4;
  return (MRL_ROWS_B_OCC3 && (SH & ~SH_TIME) != 0 && EPI_K == EPI_FVP_CACHED_B) ? 3 : 2;
}

template <int EPI_K, int SH>
__global__ __launch_bounds__(ROWS_BLOCK_B, (rows_b_occ<EPI_K, SH>())) void mlp_rows_bf16_kernel(RowsArgs a, BDims b,
                                                                       const float* __restrict__ img_g,
                                                                       const float* __restrict__ imt_g,
                                                                       const int32_t* __restrict__ skip) {
  rows_shape_b<SH>(a, b);
  constexpr bool CACHED = EPI_K == EPI_FVP_CACHED_B;
  constexpr int EPI = CACHED ? MRL_EPI_FVP : EPI_K;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const int fw = b.fwd_words;
  for (int i = threadIdx.x; i < fw / 4; i += ROWS_BLOCK_B)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
  if (EPI == MRL_EPI_FVP)
    for (int i = threadIdx.x; i < fw / 4; i += ROWS_BLOCK_B)
      reinterpret_cast<float4*>(lds + fw)[i] = reinterpret_cast<const float4*>(imt_g)[i];
  __syncthreads();
  const float* img = lds;
  const float* imt = lds + fw;
  const MlpDims dd = head_dims(a.d, b);
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
    XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, row, valid};
    float z[MAX_OUT], dz[MAX_OUT];
    float* ctile = a.cache != nullptr ? a.cache + tile * BCACHE_TILE_WORDS : nullptr;
    bf16x8 h1b[4], h2b[4];
    if constexpr (EPI == MRL_EPI_FVP) {
      if (CACHED) {
        bcache_load(ctile, 0, lane, h1b);
        bcache_load(ctile, 1, lane, h2b);
      } else {
        forward_b(img, dd, b, xl, lane, h1b, h2b, z);
      }
      jvp_b(img, imt, dd, b, xl, lane, h1b, h2b, z, dz, CACHED && a.head != MRL_HEAD_GAUSS);
    } else {
      forward_b(img, dd, b, xl, lane, h1b, h2b, z);
      if (a.cache_mode == MRL_CACHE_WRITE && ctile != nullptr) {
        bcache_store(ctile, 0, lane, h1b);
        bcache_store(ctile, 1, lane, h2b);
      }
#pragma unroll
      for (int o = 0; o < MAX_OUT; ++o) dz[o] = 0.f;
    }
    if constexpr (EPI == MRL_EPI_PPOSGD) {
      __shared__ double red[4];
      if (valid && h == 0) row_epilogue<MRL_EPI_LOSSES, MAX_OUT>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
      const double klw = wave_sum(acc1);
      if (lane == 0) red[wave] = klw;
      __syncthreads();
      const double kl = ((red[0] + red[1]) + (red[2] + red[3])) * a.inv_ng;
      RowsArgs c = a;
      c.kl_coeff = a.kl_coeff + (kl > a.kl_cutoff ? (float)(2.0 * a.cutoff_coeff * (kl - a.kl_cutoff)) : 0.f);
      double d0 = 0.0, d1 = 0.0, d2 = 0.0;
      if (valid && h == 0) row_epilogue<MRL_EPI_PPOGRAD, MAX_OUT>(c, row, z, dz, ls, sd, dls, d0, d1, d2);
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
struct VjpArgsB {
  MlpDims d;
  BDims b;
  int n_obs, gh, n_sum;
  const float* x;
  const int32_t* ept;
  double ts_limit;
  int64_t n;
  const float* ghead;
  float* slab;
  const float* cache;
};

// T tile of F tile mt from its fragments: D[row][unit] = sum over the two k-steps
__device__ inline f32x16 transpose_f(const bf16x8* fr, int mt, const bf16x8* ip) {
  f32x16 t = zero16();
  t = MFMA32B(fr[2 * mt], ip[0], t);
  t = MFMA32B(fr[2 * mt + 1], ip[1], t);
  return t;
}

typedef uint32_t vu4 __attribute__((ext_vector_type(4)));  // a 16-B register quad (asm operands)

constexpr int VJP_MAX_BLOCKS_B = 256;  // one block (4 waves) per CU at one wave per SIMD

// SH != 0: a static shape of mlp_layout.h (plain rows), every dimension a constant
template <int SH>
__device__ inline VjpArgsB vjp_shape_b(const VjpArgsB& in) {
  VjpArgsB a = in;
  if constexpr (SH != 0) {
    constexpr StaticShape S = STATIC_SHAPES[SH];
    a.d = static_dims(SH);
    a.b = bf16_dims(S.O, S.A);
    a.n_obs = S.O;
    a.n_sum = S.head == MRL_HEAD_GAUSS ? S.A : 0;
    a.gh = S.A + a.n_sum;
    a.ept = nullptr;
  }
  return a;
}

// Weight-gradient accumulators per wave (128 registers, in AGPRs: one wave per SIMD),
// written as one slab row per wave (reduced in fixed order by mrl_reduce_rows_f32).
template <bool CACHED, int SH>
__global__ __launch_bounds__(256, 1) void mlp_vjp_bf16_kernel(VjpArgsB a_in, const float* __restrict__ img_g,
                                                             const int32_t* __restrict__ skip) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // the staged cache tiles of the next tile pair (PF), 16 KB per wave
  __shared__ __attribute__((aligned(16))) bf16x8 vjp_stage[(CACHED && SH != 0) ? 4 * 2 * 2 * 4 * 64 : 1];
  if (skip != nullptr && *skip != 0) return;
  const VjpArgsB a = vjp_shape_b<SH>(a_in);
  const MlpDims& d = a.d;
  const BDims& b = a.b;
  for (int i = threadIdx.x; i < b.total_words / 4; i += 256)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
  __syncthreads();
  const float* img = lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j32 = lane & 31;
  const int A = d.A;
  const bf16x8 ip[2] = {ident_perm(0, lane), ident_perm(1, lane)};

  f32x16 gW2[2], gW1[2][2], gW0[2];  // T-tile products: [u2][o], [u1][u2], [in][u1]
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    gW2[m] = zero16();
    gW0[m] = zero16();
#pragma unroll
    for (int n = 0; n < 2; ++n) gW1[m][n] = zero16();
  }
  float gb0[2] = {0.f, 0.f}, gb1[2] = {0.f, 0.f};  // per lane = unit, this half's rows
  float gb2[MAX_OUT], gls[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    gb2[o] = 0.f;
    gls[o] = 0.f;
  }

  // Two tiles per iteration, phase by phase: the MFMA -> VALU -> MFMA dependency chain of
  // one tile (gh2 -> tanh' -> transpose -> weight-gradient products) issues between the
  // steps of the other's, so one wave per SIMD still overlaps MFMA latency.  A second tile
  // past the batch is a clamped copy of the last one with every head row masked to zero:
  // all its contributions vanish.
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * 4;
  // PF (the cached static-shape kernels, one wave per SIMD): the cache tiles of the next
  // tile pair are staged by LDS-DMA into this wave's own 16 KB of vjp_stage while this
  // pair computes (no registers held across the loop, no barrier: a wave reads only what
  // it staged); read back by inline-asm ds_reads, which the compiler's LDS-DMA alias
  // tracking cannot turn into vmcnt(0) drains in front of the image reads.
  constexpr bool PF = CACHED && SH != 0;
  auto tile_of = [&](int64_t t0, int u) {
    const int64_t tu = t0 + u * stride;
    return tu < ntiles ? tu : ntiles - 1;
  };
  bf16x8* const stg = vjp_stage + wave * (2 * 2 * 4 * 64);  // [u][layer][s][lane]
  auto dma_pair = [&](int64_t t0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(a.cache + tile_of(t0, u) * BCACHE_TILE_WORDS);
#pragma unroll
      for (int f = 0; f < 8; ++f)  // f = layer * 4 + s
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + f * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(stg + (u * 8 + f) * 64), 16, 0, 0);
    }
  };
  // the pair's input and head rows: every load unconditional from a clamped address
  // (static n_obs / A / n_sum), issued together one pair ahead, validity applied as 0 / 1
  // factors at use (a select on a loaded value becomes a branch and a vmcnt(0) drain)
  float xr[2][8 * MAX_KS0B], gr_[2][8], glr[2][MAX_OUT];
  auto load_rows = [&](int64_t t0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t row = tile_of(t0, u) * 32 + j32;
      const int64_t rc = row < a.n ? row : 0;
      const float* xp = a.x + rc * a.n_obs;
#pragma unroll
      for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int k = 16 * s0 + 8 * h + jj;
          xr[u][8 * s0 + jj] = s0 < b.KS0B ? xp[k < a.n_obs ? k : a.n_obs - 1] : 0.f;
        }
      const float* gp = a.ghead + rc * a.gh;
#pragma unroll
      for (int o = 0; o < 8; ++o) gr_[u][o] = gp[o < A ? o : A - 1];
#pragma unroll
      for (int q = 0; q < MAX_OUT; ++q) glr[u][q] = q < a.n_sum ? gp[A + q] : 0.f;
    }
  };
  if constexpr (PF) {
    const int64_t t0 = (int64_t)blockIdx.x * 4 + wave;
    if (t0 < ntiles) {
      load_rows(t0);
      dma_pair(t0);
    }
  }
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += 2 * stride) {
    bf16x8 h1b[2][4], h2b[2][4], gB[2], xb[2][MAX_KS0B];
    bool live[2];
    if constexpr (PF) {
      // this pair's staged tiles: own DMA landed -> registers -> the next pair's DMA
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(stg) + 16 * lane;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sI = 0; sI < 4; ++sI) {
          vu4 v1, v2;
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v1) : "v"(base), "i"(((u * 8 + sI) * 64) * 16));
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v2) : "v"(base), "i"(((u * 8 + 4 + sI) * 64) * 16));
          h1b[u][sI] = __builtin_bit_cast(bf16x8, v1);
          h2b[u][sI] = __builtin_bit_cast(bf16x8, v2);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(h1b[0][0]), "+v"(h1b[0][1]), "+v"(h1b[0][2]), "+v"(h1b[0][3]),
                   "+v"(h1b[1][0]), "+v"(h1b[1][1]), "+v"(h1b[1][2]), "+v"(h1b[1][3]), "+v"(h2b[0][0]),
                   "+v"(h2b[0][1]), "+v"(h2b[0][2]), "+v"(h2b[0][3]), "+v"(h2b[1][0]), "+v"(h2b[1][1]),
                   "+v"(h2b[1][2]), "+v"(h2b[1][3])::"memory");
    }
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t tu = tile + u * stride;
        live[u] = tu < ntiles;
        const int64_t row = (live[u] ? tu : ntiles - 1) * 32 + j32;
        float fv = (live[u] && row < a.n && h == 0) ? 1.f : 0.f, fx = row < a.n ? 1.f : 0.f;
        asm volatile("" : "+v"(fv), "+v"(fx));
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const float g = o < A ? gr_[u][o] * fv : 0.f;
          gb2[o] += g;
          gB[u][o] = (__bf16)g;
        }
#pragma unroll
        for (int q = 0; q < MAX_OUT; ++q) gls[q] += q < a.n_sum ? glr[u][q] * fv : 0.f;
#pragma unroll
        for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int k = 16 * s0 + 8 * h + jj;
            xb[u][s0][jj] = (__bf16)((s0 < b.KS0B && k < a.n_obs) ? xr[u][8 * s0 + jj] * fx : 0.f);
          }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if constexpr (PF) break;
      const int64_t tu = tile + u * stride;
      live[u] = tu < ntiles;
      const int64_t tc = live[u] ? tu : ntiles - 1;
      const int64_t row = tc * 32 + j32;
      const bool valid = live[u] && row < a.n;
      XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, row, row < a.n};
      if constexpr (CACHED) {
        bcache_load(a.cache + tc * BCACHE_TILE_WORDS, 1, lane, h2b[u]);
        bcache_load(a.cache + tc * BCACHE_TILE_WORDS, 0, lane, h1b[u]);
      } else {
        float zz[MAX_OUT];
        forward_b(img, head_dims(d, b), b, xl, lane, h1b[u], h2b[u], zz);
      }
#pragma unroll
      for (int s0 = 0; s0 < MAX_KS0B; ++s0) xb[u][s0] = s0 < b.KS0B ? x_frag(xl, s0, h) : bf16x8{};
      // head-gradient row (f32) and its bf16 operand: o = 8h + j (h = 1: zero, A <= 8)
      const float* gr = a.ghead + (row < a.n ? row : 0) * a.gh;
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const float g = (valid && h == 0 && o < A) ? gr[o] : 0.f;
        gb2[o] += g;
        gB[u][o] = (__bf16)g;
      }
#pragma unroll
      for (int q = 0; q < MAX_OUT; ++q) gls[q] += (valid && h == 0 && q < a.n_sum) ? gr[A + q] : 0.f;
    }
    if constexpr (PF) {  // the next pair's rows and cache tiles, under this pair's MFMAs
      if (tile + 2 * stride < ntiles) {
        load_rows(tile + 2 * stride);
        dma_pair(tile + 2 * stride);
      }
    }
    // gh2 = W2 . G (F layout), ga2 = gh2 (1 - h2^2)
    bf16x8 ga2b[2][4];
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) {
      f32x16 g2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) g2[u] = MFMA32B(frag_at(img, b.bw2, mo, lane), gB[u], zero16());
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f32x16 h2 = unpack16(h2b[u], mo);
#pragma unroll
        for (int r = 0; r < 16; ++r) g2[u][r] *= dtanh(h2[r]);
        ga2b[u][2 * mo] = pack8(g2[u], 0);
        ga2b[u][2 * mo + 1] = pack8(g2[u], 1);
      }
    }
    // gW2 += H2^T G
    {
      f32x16 gT[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) gT[u] = MFMA32B(gB[u], ident_nat(0, lane), zero16());  // D[row][o]
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        f32x16 h2T[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) h2T[u] = transpose_f(h2b[u], m, ip);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          gW2[m] = MFMA32B(pack8(h2T[u], 0), pack8(gT[u], 0), gW2[m]);
          gW2[m] = MFMA32B(pack8(h2T[u], 1), pack8(gT[u], 1), gW2[m]);
        }
      }
    }
    // ga2 and the inputs in T layout
    bf16x8 ga2T[2][2][2], xT[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      f32x16 t[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) t[u] = transpose_f(ga2b[u], m, ip);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) gb1[m] += t[u][r];
        ga2T[u][m][0] = pack8(t[u], 0);
        ga2T[u][m][1] = pack8(t[u], 1);
      }
    }
    {
      f32x16 t[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        t[u] = zero16();
#pragma unroll
        for (int s0 = 0; s0 < MAX_KS0B; ++s0)
          if (s0 < b.KS0B) t[u] = MFMA32B(xb[u][s0], ident_nat(16 * s0, lane), t[u]);  // D[row][in]
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        xT[u][0] = pack8(t[u], 0);
        xT[u][1] = pack8(t[u], 1);
      }
    }
    // per u1 tile: gh1 (T layout) = ga2^T . W1^T, ga1 = gh1 (1 - h1^2), then
    // gW1 += H1^T GA2 and gW0 += X^T GA1
#pragma unroll
    for (int no = 0; no < 2; ++no) {
      f32x16 ga1[2], h1T[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) ga1[u] = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u) ga1[u] = MFMA32B(ga2b[u][s], frag_at(img, b.bt1, no * 4 + s, lane), ga1[u]);
#pragma unroll
      for (int u = 0; u < 2; ++u) h1T[u] = transpose_f(h1b[u], no, ip);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          ga1[u][r] *= dtanh(h1T[u][r]);
          gb0[no] += ga1[u][r];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const bf16x8 h1p = pack8(h1T[u], sp);
          gW1[no][0] = MFMA32B(h1p, ga2T[u][0][sp], gW1[no][0]);
          gW1[no][1] = MFMA32B(h1p, ga2T[u][1][sp], gW1[no][1]);
          gW0[no] = MFMA32B(xT[u][sp], pack8(ga1[u], sp), gW0[no]);
        }
    }
    (void)live;
  }

  // per-wave partial gradient in flat theta layout; accumulator tiles are D[i][j] with
  // j = lane & 31 and i = cperm(r, h)
  float* out = a.slab + ((int64_t)blockIdx.x * 4 + wave) * d.P;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = cperm(r, h);
      if (i < d.O) out[d.tW0 + i * HID + 32 * m + j32] = gW0[m][r];
      if (j32 < A) out[d.tW2 + (32 * m + i) * A + j32] = gW2[m][r];
#pragma unroll
      for (int n = 0; n < 2; ++n) out[d.tW1 + (32 * m + i) * HID + 32 * n + j32] = gW1[m][n][r];
    }
  // bias sums: this half's rows, then the other half's (lanes l, l ^ 32 hold one unit)
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const float s0 = xor32_add(gb0[m]);
    const float s1 = xor32_add(gb1[m]);
    if (h == 0) {
      out[d.tb0 + 32 * m + j32] = s0;
      out[d.tb1 + 32 * m + j32] = s1;
    }
  }
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    const float sum = wave_sumf(gb2[o]);
    if (lane == 0 && o < A) out[d.tb2 + o] = sum;
  }
  for (int q = 0; q < a.n_sum; ++q) {
    const float sum = wave_sumf(gls[q]);
    if (lane == 0) out[d.tls + q] = sum;
  }
}

}  // namespace mrl

using namespace mrl;

static int check_desc_b(const mrl_mlp_desc* d) {
  if (d == nullptr) return fail(E_ARG, "null mlp desc");
  if (d->n_hidden != HID || d->n_layers != 2)
    return fail(E_UNSUPPORTED, "only hid_sizes=[64,64] is implemented on the fused HIP path");
  if (d->n_in < 1 || d->n_in > MAX_IN) return fail(E_UNSUPPORTED, "n_in must be in [1, 32]");
  if (d->n_out < 1 || d->n_out > MAX_OUT) return fail(E_UNSUPPORTED, "n_out must be in [1, 8]");
  if (d->head < 0 || d->head > 2) return fail(E_ARG, "bad head kind");
  if (d->head == MRL_HEAD_LINEAR && d->n_out != 1) return fail(E_ARG, "linear head needs n_out=1");
  if (d->cus < 0 || d->cus > 1024) return fail(E_ARG, "cus must be in [0, 1024]");
  return OK;
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid caps, swept with tools/fvp_probe.py at 4.19 M rows (MRL_ROWS_BF16_BLOCKS
// overrides both): the Fisher-product JVP (154 VGPRs: 3 blocks per CU) is fastest at
// exactly one resident round (768: 0.347 ms; 1024: 0.47, 1536: 0.356, 2048: 0.395);
// the forward passes (≤ 128 VGPRs) at three rounds and more (3072: surrgrad 0.526,
// prob 0.299 ms; 2048: 0.538 / 0.303).
constexpr int ROWS_FVP_BLOCKS_B = 768;
// caps per 256 CUs, scaled by the desc's `cus` (mlp_kernels.hip desc_cus)
static int64_t desc_cus_b(const mrl_mlp_desc* d) { return d != nullptr && d->cus > 0 ? d->cus : 256; }
static int64_t scaled_cap(int64_t cap, int64_t cus) { return cap * cus / 256 > 0 ? cap * cus / 256 : 1; }
static int64_t rows_blocks_b(int64_t n, bool fvp = false, int64_t cus = 256) {
  static const int64_t env_cap = [] {
    const char* e = getenv("MRL_ROWS_BF16_BLOCKS");
    return (int64_t)(e ? atoi(e) : 0);
  }();
  const int64_t cap = env_cap > 0 ? env_cap : scaled_cap(fvp ? ROWS_FVP_BLOCKS_B : ROWS_MAX_BLOCKS_B, cus);
  int64_t g = cdiv(cdiv(n, 32), 4);
  if (g < 1) g = 1;
  return g > cap ? cap : g;
}
static int64_t vjp_blocks_b(int64_t n, int64_t cus = 256) {
  int64_t g = cdiv(cdiv(n, 32), 4);
  if (g < 1) g = 1;
  const int64_t cap = scaled_cap(VJP_MAX_BLOCKS_B, cus);
  return g > cap ? cap : g;
}

extern "C" {

int64_t mrl_mlp_image_words_bf16(const mrl_mlp_desc* d) {
  if (check_desc_b(d) != OK) return -1;
  return bf16_dims(d->n_in, d->n_out).total_words;
}
int64_t mrl_act_cache_words_bf16(int64_t n) { return cdiv(n, 32) * BCACHE_TILE_WORDS; }
int64_t mrl_partial_rows_bf16(int64_t n) { return rows_blocks_b(n) * 4; }
int64_t mrl_slab_rows_bf16(int64_t n) { return vjp_blocks_b(n) * 4; }
int64_t mrl_mlp_partial_rows_bf16(const mrl_mlp_desc* d, int64_t n) {
  if (check_desc_b(d) != OK) return -1;
  return rows_blocks_b(n, false, desc_cus_b(d)) * 4;
}
int64_t mrl_mlp_slab_rows_bf16(const mrl_mlp_desc* d, int64_t n) {
  if (check_desc_b(d) != OK) return -1;
  return vjp_blocks_b(n, desc_cus_b(d)) * 4;
}

int mrl_mlp_pack_bf16(const mrl_mlp_desc* d, const float* theta, float* image, int32_t fwd_only,
                      const int32_t* skip, void* stream) {
  int rc = check_desc_b(d);
  if (rc) return rc;
  if (!theta || !image) return fail(E_ARG, "null pointer");
  const MlpDims m = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  const BDims b = bf16_dims(d->n_in, d->n_out);
  const int words = fwd_only ? b.fwd_words : b.total_words;
  hipLaunchKernelGGL(mlp_pack_bf16_kernel, dim3((words + 255) / 256), dim3(256), 0, (hipStream_t)stream, m, b, theta,
                     image, words, skip);
  return hip_check(hipGetLastError(), "mrl_mlp_pack_bf16");
}

int mrl_mlp_rows_bf16(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image,
                      const float* tangent, const float* image_t, const mrl_rows_io* io, const int32_t* skip,
                      void* stream) {
  int rc = check_desc_b(d);
  if (rc) return rc;
  if (!io || !image || !io->x) return fail(E_ARG, "null pointer");
  if (io->n <= 0) return OK;
  RowsArgs a{};
  a.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
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
  const BDims b = bf16_dims(d->n_in, d->n_out);
  const size_t shm = (size_t)b.fwd_words * 4 * (epi == MRL_EPI_FVP ? 2 : 1);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(epi == MRL_EPI_PPOSGD ? 1 : rows_blocks_b(io->n, epi == MRL_EPI_FVP, io->partial != nullptr ? desc_cus_b(d) : 256)),
      blk(ROWS_BLOCK_B);
  // the benchmark nets as static shapes (plain rows; a time-feature column built from
  // ep_t takes the generic kernel); policy epilogues only for the policy shapes
  int sh = 0;
  if (!io->ep_t)
    for (int i = 1; i < N_STATIC_SHAPES; ++i)
      if (STATIC_SHAPES[i].O == d->n_in && STATIC_SHAPES[i].A == d->n_out && STATIC_SHAPES[i].head == d->head) sh = i;
  // the value nets' prediction pass reads the time feature from ep_t (SH_TIME variants)
  int sht = 0;
  if (io->ep_t && epi == MRL_EPI_PROB && d->head == MRL_HEAD_LINEAR)
    for (int i = 3; i <= 4; ++i)
      if (STATIC_SHAPES[i].O == d->n_in && STATIC_SHAPES[i].A == d->n_out) sht = i | SH_TIME;
  const bool pol = sh == 1 || sh == 2, vf = sh == 3 || sh == 4;
#define MRL_ROWSB(EK, OK)                                                                                          \
  do {                                                                                                             \
    if ((OK) && sh == 1) hipLaunchKernelGGL((mlp_rows_bf16_kernel<EK, 1>), grid, blk, shm, s, a, b, image, image_t, skip); \
    else if ((OK) && sh == 2) hipLaunchKernelGGL((mlp_rows_bf16_kernel<EK, 2>), grid, blk, shm, s, a, b, image, image_t, skip); \
    else if ((OK) && sh == 3) hipLaunchKernelGGL((mlp_rows_bf16_kernel<EK, 3>), grid, blk, shm, s, a, b, image, image_t, skip); \
    else if ((OK) && sh == 4) hipLaunchKernelGGL((mlp_rows_bf16_kernel<EK, 4>), grid, blk, shm, s, a, b, image, image_t, skip); \
    else hipLaunchKernelGGL((mlp_rows_bf16_kernel<EK, 0>), grid, blk, shm, s, a, b, image, image_t, skip);               \
  } while (0)
  switch (epi) {
    case MRL_EPI_PROB:
      if (sht == (3 | SH_TIME)) hipLaunchKernelGGL((mlp_rows_bf16_kernel<MRL_EPI_PROB, 3 | SH_TIME>), grid, blk, shm, s, a, b, image, image_t, skip);
      else if (sht == (4 | SH_TIME)) hipLaunchKernelGGL((mlp_rows_bf16_kernel<MRL_EPI_PROB, 4 | SH_TIME>), grid, blk, shm, s, a, b, image, image_t, skip);
      else MRL_ROWSB(MRL_EPI_PROB, true);
      break;
    case MRL_EPI_LOSSES: MRL_ROWSB(MRL_EPI_LOSSES, pol); break;
    case MRL_EPI_SURRGRAD: MRL_ROWSB(MRL_EPI_SURRGRAD, pol); break;
    case MRL_EPI_VFLOSS: MRL_ROWSB(MRL_EPI_VFLOSS, vf); break;
    case MRL_EPI_FVP:
      if (a.cache_mode == MRL_CACHE_READ) MRL_ROWSB(EPI_FVP_CACHED_B, pol);
      else MRL_ROWSB(MRL_EPI_FVP, pol);
      break;
    case MRL_EPI_PPOGRAD: MRL_ROWSB(MRL_EPI_PPOGRAD, pol); break;
    case MRL_EPI_PPOSGD: MRL_ROWSB(MRL_EPI_PPOSGD, pol); break;
  }
#undef MRL_ROWSB
  return hip_check(hipGetLastError(), "mrl_mlp_rows_bf16");
}

int mrl_mlp_vjp_bf16(const mrl_mlp_desc* d, const float* image, const float* x, const int32_t* ep_t, double ts_limit,
                     const float* ghead, int64_t n, float* slab, const float* act_cache, const int32_t* skip,
                     void* stream) {
  int rc = check_desc_b(d);
  if (rc) return rc;
  if (!image || !x || !ghead || !slab) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  VjpArgsB a{};
  a.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  a.b = bf16_dims(d->n_in, d->n_out);
  a.n_obs = d->n_in - (ep_t ? 1 : 0);
  a.n_sum = d->head == MRL_HEAD_GAUSS ? d->n_out : 0;
  a.gh = d->n_out + a.n_sum;
  a.x = x;
  a.ept = ep_t;
  a.ts_limit = ts_limit;
  a.n = n;
  a.ghead = ghead;
  a.slab = slab;
  a.cache = act_cache;
  const size_t shm = (size_t)a.b.total_words * 4;
  const dim3 grid(vjp_blocks_b(n, desc_cus_b(d))), blk(256);
  hipStream_t s = (hipStream_t)stream;
  // the benchmark policies and value nets as static shapes (plain rows only: the VF
  // fit reads its materialised [obs, t / limit] rows; a time feature built from ep_t
  // takes the generic kernel, which spills at the VF's shape)
  int sh = 0;
  if (!ep_t)
    for (int i = 1; i < N_STATIC_SHAPES; ++i)
      if (STATIC_SHAPES[i].O == d->n_in && STATIC_SHAPES[i].A == d->n_out && STATIC_SHAPES[i].head == d->head) sh = i;
#define MRL_VJPB(C)                                                                                              \
  do {                                                                                                           \
    if (sh == 1) hipLaunchKernelGGL((mlp_vjp_bf16_kernel<C, 1>), grid, blk, shm, s, a, image, skip);              \
    else if (sh == 2) hipLaunchKernelGGL((mlp_vjp_bf16_kernel<C, 2>), grid, blk, shm, s, a, image, skip);         \
    else if (sh == 3) hipLaunchKernelGGL((mlp_vjp_bf16_kernel<C, 3>), grid, blk, shm, s, a, image, skip);         \
    else if (sh == 4) hipLaunchKernelGGL((mlp_vjp_bf16_kernel<C, 4>), grid, blk, shm, s, a, image, skip);         \
    else hipLaunchKernelGGL((mlp_vjp_bf16_kernel<C, 0>), grid, blk, shm, s, a, image, skip);                      \
  } while (0)
  if (act_cache != nullptr) MRL_VJPB(true);
  else MRL_VJPB(false);
#undef MRL_VJPB
  return hip_check(hipGetLastError(), "mrl_mlp_vjp_bf16");
}

}  // extern "C"
