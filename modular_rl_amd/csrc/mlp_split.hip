// fp32-accurate Fisher-vector product on bf16 MFMA: split operands.
//
// The TRPO update spends ~90 % of its time in the ten Fisher products of CG
// (trpo.py:45-58, 86-92: fvp = grad(grad(kl_ff) . v)).  On gfx950 the exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate, and the f32 pair of kernels
// (mlp_kernels.hip) sits at the f32 MFMA floor of the chip's power-held clock.  Here every
// f32 MFMA operand v is split exactly into three bf16 parts, v = v0 + v1 + v2 (RNE
// splits: v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1); each subtraction is
// exact and the last remainder has at most 8 significant bits), and a product a.b is
// the sum of the part products a_i.b_j on v_mfma_f32_32x32x16_bf16 with f32 accumulation:
//   NPROD = 9: all nine products -- every a_i.b_j is exact in f32, so a.b is formed
//              exactly and the only rounding is the f32 accumulation, as in the f32 MFMA;
//   NPROD = 6: drops a1.b2, a2.b1, a2.b2 (each <= 2^-25 |a.b|, below one f32 ulp).
// The parts are accumulated smallest first, 16 k-terms per MFMA (fewer roundings than a
// per-product f32 fma chain).  So this is fp32 arithmetic in its accuracy -- checked
// against the float64 oracle at the same 1e-4 and against the exact-f32 kernels to f32
// rounding (tests/test_gpu_split.py) -- on the bf16 matrix cores.
//
// Layouts are those of the bf16 mode (bf16_frag.h, mlp_bf16.hip header): F tiles
// D[unit][row] chain as B fragments; the split image is the bf16 image's f32 section
// (biases, VALU head) followed by three copies of its bf16 section, part p at +p * PS.
// The primal activations come from the f32 activation cache of the update's SURRGRAD
// pass (mlp_kernels.hip cache layout = the F-tile register order), split on load.
#include <math.h>
#include <stdlib.h>

#include "../../include/mrl_hip.h"
#include "bf16_frag.h"
#include "mlp_device.h"
#include "rows_epilogue.h"

namespace mrl {

// Split image: the f32 section [0, fa0), then the three parts of the forward fragments
// (fa0, fa1: FW words each, part p of a forward segment at its bf16-image offset + p FW),
// then the three parts of the backward fragments (bw2, bt1: BW words each, part p at its
// bf16-image offset + 2 FW + p BW).  A pass that needs only the forward segments (the JVP,
// the tangent's image) stages the first fa0 + 3 FW words.
__host__ __device__ constexpr int split_fw(const BDims& b) { return b.fwd_words - b.fa0; }
__host__ __device__ constexpr int split_bw(const BDims& b) { return b.total_words - b.fwd_words; }
__host__ __device__ constexpr int split_fwd_words(const BDims& b) { return b.fa0 + 3 * split_fw(b); }
__host__ __device__ constexpr int split_image_words(const BDims& b) { return split_fwd_words(b) + 3 * split_bw(b); }
// offset of part 0 of a backward segment (bw2 / bt1 of the bf16 image)
__host__ __device__ constexpr int split_bwd_seg(const BDims& b, int seg) { return seg + 2 * split_fw(b); }

// part p (0, 1, 2) of an f32 value's exact three-way bf16 split
__device__ inline float bf16_part(float v, int p) {
  const __bf16 a = (__bf16)v;
  if (p == 0) return (float)a;
  const float r = v - (float)a;
  const __bf16 c = (__bf16)r;
  if (p == 1) return (float)c;
  return r - (float)c;
}

__global__ void mlp_pack_split_kernel(MlpDims d, BDims b, const float* __restrict__ th, float* __restrict__ image,
                                      int words, const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  if (w < b.fa0) {  // f32 section: biases and the VALU head, the bf16 image's order
    int idx;
    if (w < b.fb1) idx = d.fb0 + (w - b.fb0);
    else if (w < b.hv) idx = d.fb1 + (w - b.fb1);
    else if (w < b.hb) idx = d.hv + (w - b.hv);
    else idx = d.hb + (w - b.hb);
    image[w] = image_value(d, th, idx);
    return;
  }
  const int FW = split_fw(b), BW = split_bw(b), f0 = split_fwd_words(b);
  const int part = w < f0 ? (w - b.fa0) / FW : (w - f0) / BW;
  const int wp = w < f0 ? b.fa0 + (w - b.fa0) % FW : b.fwd_words + (w - f0) % BW;
  int seg, rel;
  if (wp < b.fa1) { seg = 0; rel = wp - b.fa0; }
  else if (wp < b.bw2) { seg = 1; rel = wp - b.fa1; }
  else if (wp < b.bt1) { seg = 2; rel = wp - b.bw2; }
  else { seg = 3; rel = wp - b.bt1; }
  const int frag = rel >> 2, q = rel & 3;
  const __bf16 lo = (__bf16)bf16_part(bimage_elem(d, b, th, seg, frag, 2 * q), part);
  const __bf16 hi = (__bf16)bf16_part(bimage_elem(d, b, th, seg, frag, 2 * q + 1), part);
  const uint32_t v = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
  image[w] = __uint_as_float(v);
}

// The exact three-way split of 8 values, two at a time: one v_cvt_pk_bf16_f32 per part
// pair, the widening and the remainders on packed f32 (v_pk_add_f32) -- the same RNE
// conversions and exact subtractions as the element-wise form, about 4.5 VALU per value
// instead of 7 (the split is most of these kernels' VALU work).  Explicit vector types, so
// the packing does not depend on the SLP vectoriser.
// (split2: mlp_device.h)
__device__ inline void split8v(const float* v, bf16x8* out) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    bf16x2 a, c, e;
    split2(f32x2{v[j], v[j + 1]}, a, c, e);
    out[0][j] = a[0];
    out[0][j + 1] = a[1];
    out[1][j] = c[0];
    out[1][j + 1] = c[1];
    out[2][j] = e[0];
    out[2][j + 1] = e[1];
  }
}
// the three parts of registers 8 sp .. 8 sp + 7 of an F tile (the B fragment pack8 forms)
__device__ inline void split8(const f32x16& t, int sp, bf16x8* out) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = t[8 * sp + j];
  split8v(v, out);
}

// acc += W . X for one k-step: W = the image fragment f of segment `seg` (parts at
// +p * PS), X = three parts; smallest products first
template <int NPROD>
__device__ inline void mfma_split(const float* img, int seg, int PS, int f, int lane, const bf16x8* x, f32x16& acc) {
  const bf16x8 w0 = frag_at(img, seg, f, lane), w1 = frag_at(img, seg + PS, f, lane);
  const bf16x8 w2 = frag_at(img, seg + 2 * PS, f, lane);
  if constexpr (NPROD == 9) {
    acc = MFMA32B(w2, x[2], acc);
    acc = MFMA32B(w2, x[1], acc);
    acc = MFMA32B(w1, x[2], acc);
  }
  acc = MFMA32B(w2, x[0], acc);
  acc = MFMA32B(w0, x[2], acc);
  acc = MFMA32B(w1, x[1], acc);
  acc = MFMA32B(w1, x[0], acc);
  acc = MFMA32B(w0, x[1], acc);
  acc = MFMA32B(w0, x[0], acc);
}

#ifndef MRL_SPLIT_NPROD
#define MRL_SPLIT_NPROD 6
#endif
// scheduling fences between the passes' phases (0: let the compiler interleave one
// phase's VALU splits with the previous phase's MFMAs)
#ifndef MRL_SPLIT_FENCES
#define MRL_SPLIT_FENCES 1
#endif
#if MRL_SPLIT_FENCES
#define VJP_SPLIT_FENCE() __builtin_amdgcn_sched_barrier(0)
#define FVP_SPLIT_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define VJP_SPLIT_FENCE() ((void)0)
#define FVP_SPLIT_FENCE() ((void)0)
#endif

template <int SH>
__device__ inline void split_shape(RowsArgs& a, BDims& b) {
  if constexpr (SH != 0) {
    constexpr StaticShape S = STATIC_SHAPES[SH];
    a.d = static_dims(SH);
    a.A = S.A;
    a.head = S.head;
    a.n_obs = S.O;
    a.gh = S.head == MRL_HEAD_GAUSS ? 2 * S.A : S.A;
    a.ept = nullptr;
    b = bf16_dims(S.O, S.A);
  }
}

// waves per block of the JVP rows kernel: 4 (two blocks per CU at 2 waves per SIMD: the
// staged images take 67 KB of LDS per block) or 12 (one block per CU at 3 waves per SIMD)
#ifndef MRL_SPLIT_ROWS_WAVES
#define MRL_SPLIT_ROWS_WAVES 4
#endif
constexpr int SPLIT_ROWS_WAVES = MRL_SPLIT_ROWS_WAVES;
constexpr int SPLIT_ROWS_BLOCK = 64 * SPLIT_ROWS_WAVES;

// The Fisher product's forward half (trpo.py:45-58): JVP of the head along the tangent
// from the cached f32 h1 / h2, then the KL-metric head-gradient rows (row_epilogue FVP),
// exactly what mlp_rows_kernel<EPI_FVP_CACHED> computes, with split-operand products.
#ifndef MRL_SPLIT_FVP_OCC  // waves per SIMD the JVP rows kernel is compiled for
#define MRL_SPLIT_FVP_OCC 2
#endif
template <int SH>
__global__ __launch_bounds__(SPLIT_ROWS_BLOCK, (4 * MRL_SPLIT_FVP_OCC / SPLIT_ROWS_WAVES > 0
                                                 ? 4 * MRL_SPLIT_FVP_OCC / SPLIT_ROWS_WAVES : 1))
    void mlp_fvp_split_kernel(RowsArgs a, BDims b,
                                                                           const float* __restrict__ img_g,
                                                                           const float* __restrict__ imt_g,
                                                                           const int32_t* __restrict__ skip) {
  split_shape<SH>(a, b);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const int W = split_fwd_words(b), PS = split_fw(b);  // forward segments only
  for (int i = threadIdx.x; i < W / 4; i += SPLIT_ROWS_BLOCK) {
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
    reinterpret_cast<float4*>(lds + W)[i] = reinterpret_cast<const float4*>(imt_g)[i];
  }
  __syncthreads();
  const float* img = lds;
  const float* imt = lds + W;
  const MlpDims dd = head_dims(a.d, b);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile indices
  const int A = a.A;
  float ls[MAX_OUT], sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
  for (int j = 0; j < MAX_OUT; ++j) {
    ls[j] = (a.logstd != nullptr && j < A) ? a.logstd[j] : 0.f;
    sd[j] = expf(ls[j]);
    dls[j] = (a.dlogstd != nullptr && j < A) ? a.dlogstd[j] : 0.f;
  }
  const bool need_z = a.head != MRL_HEAD_GAUSS;  // the DiagGauss metric does not use the mean
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * SPLIT_ROWS_WAVES;
  // Software pipeline (SQ, round 4: 0.39 of the wave time parked on s_waitcnt): a tile's
  // inputs x and h1 are loaded during the previous tile; at a tile's start its h2 loads
  // are issued first, then the next tile's x / h1 (vmcnt retires in order, so the wait
  // for h2 before the head leaves the prefetch in flight)
  int64_t tile = (int64_t)blockIdx.x * SPLIT_ROWS_WAVES + wave;
  float xv[MAX_KS0B][8];
  f32x16 h1[2];
  auto load_xh1 = [&](int64_t t, float (&x)[MAX_KS0B][8], f32x16* hh) {
    const int64_t r = t * 32 + (lane & 31);
    XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, r, r < a.n};
#pragma unroll
    for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[s0][j] = s0 < b.KS0B ? xl(16 * s0 + 8 * h + j) : 0.f;
    cache_load(a.cache + t * CACHE_TILE_FLOATS, lane, 0, hh[0]);
    cache_load(a.cache + t * CACHE_TILE_FLOATS, lane, 1, hh[1]);
  };
  if (tile < ntiles) load_xh1(tile, xv, h1);
  for (; tile < ntiles; tile += stride) {
    const int64_t row = tile * 32 + (lane & 31);
    const bool valid = row < a.n;
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
    f32x16 h2[2];
    cache_load(ct, lane, 2, h2[0]);
    cache_load(ct, lane, 3, h2[1]);
    __builtin_amdgcn_sched_barrier(0);
    const int64_t tn = tile + stride < ntiles ? tile + stride : tile;  // the last tile re-reads itself
    float xn[MAX_KS0B][8];
    f32x16 h1n[2];
    load_xh1(tn, xn, h1n);
    __builtin_amdgcn_sched_barrier(0);
    f32x16 dh[2];
    // layer 0 tangent: dh = (x dW0 + db0) (1 - h1^2)
    dh[0] = load_bias16(imt, b.fb0, 0, h);
    dh[1] = load_bias16(imt, b.fb0, 1, h);
#pragma unroll
    for (int s0 = 0; s0 < MAX_KS0B; ++s0) {
      if (s0 < b.KS0B) {
        bf16x8 xs[3];
        split8v(xv[s0], xs);
        mfma_split<MRL_SPLIT_NPROD>(imt, b.fa0, PS, 0 * b.KS0B + s0, lane, xs, dh[0]);
        mfma_split<MRL_SPLIT_NPROD>(imt, b.fa0, PS, 1 * b.KS0B + s0, lane, xs, dh[1]);
      }
    }
    mul_dtanh16(dh[0], h1[0]);
    mul_dtanh16(dh[1], h1[1]);
    // layer 1 tangent: da = (dh W1 + h1 dW1 + db1) (1 - h2^2); each input fragment is
    // split once and feeds both output tiles (per tile the k order is unchanged: the four
    // dh fragments, then the four h1 fragments)
    float z[MAX_OUT], dz[MAX_OUT], dzt[MAX_OUT];
#pragma unroll
    for (int o = 0; o < MAX_OUT; ++o) z[o] = dz[o] = dzt[o] = 0.f;
    f32x16 da2[2] = {load_bias16(imt, b.fb1, 0, h), load_bias16(imt, b.fb1, 1, h)};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 ps[3];
      split8(dh[s >> 1], s & 1, ps);
      mfma_split<MRL_SPLIT_NPROD>(img, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
      mfma_split<MRL_SPLIT_NPROD>(img, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
    }
    FVP_SPLIT_FENCE();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 ps[3];
      split8(h1[s >> 1], s & 1, ps);
      mfma_split<MRL_SPLIT_NPROD>(imt, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
      mfma_split<MRL_SPLIT_NPROD>(imt, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
    }
    FVP_SPLIT_FENCE();
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) {
      f32x16& da = da2[mo];
      mul_dtanh16(da, h2[mo]);
      // the head on the f32 VALU: dz = da . W2 + h2 . dW2 (+ db2 in head_finish), z = h2 . W2
      if (need_z) head_partial_mt(img, dd, h2[mo], mo, h, z);
      head_partial_mt(img, dd, da, mo, h, dz);
      head_partial_mt(imt, dd, h2[mo], mo, h, dzt);
      FVP_SPLIT_FENCE();
    }
    if (need_z) head_finish(img, dd, z);
#pragma unroll
    for (int o = 0; o < MAX_OUT; ++o) dz[o] += dzt[o];
    head_finish(imt, dd, dz);
    if (valid && h == 0) row_epilogue<MRL_EPI_FVP, MAX_OUT>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
#pragma unroll
    for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[s0][j] = xn[s0][j];
    h1[0] = h1n[0];
    h1[1] = h1n[1];
  }
  (void)acc0;
  (void)acc1;
  (void)acc2;
}


// ------------------------------------------------------------------ VJP
// acc += A . B over the split parts of both operands (A[p], B[p]: part p), smallest first
template <int NPROD>
__device__ inline void mma_split(const bf16x8* A, const bf16x8* B, f32x16& acc) {
  if constexpr (NPROD == 9) {
    acc = MFMA32B(A[2], B[2], acc);
    acc = MFMA32B(A[2], B[1], acc);
    acc = MFMA32B(A[1], B[2], acc);
  }
  acc = MFMA32B(A[2], B[0], acc);
  acc = MFMA32B(A[0], B[2], acc);
  acc = MFMA32B(A[1], B[1], acc);
  acc = MFMA32B(A[1], B[0], acc);
  acc = MFMA32B(A[0], B[1], acc);
  acc = MFMA32B(A[0], B[0], acc);
}

struct VjpSplitArgs {
  MlpDims d;
  BDims b;
  int n_obs, gh, n_sum;
  const float* x;
  int64_t n;
  const float* ghead;
  float* slab;
  const float* cache;
};

template <int SH>
__device__ inline VjpSplitArgs vjp_shape_s(const VjpSplitArgs& in) {
  VjpSplitArgs a = in;
  if constexpr (SH != 0) {
    constexpr StaticShape S = STATIC_SHAPES[SH];
    a.d = static_dims(SH);
    a.b = bf16_dims(S.O, S.A);
    a.n_obs = S.O;
    a.n_sum = S.head == MRL_HEAD_GAUSS ? S.A : 0;
    a.gh = S.A + a.n_sum;
  }
  return a;
}

// T tile (D[row][unit]) of the F tile whose two fragments are f0 (registers 0-7) and f1
__device__ inline f32x16 transpose_ff(const bf16x8& f0, const bf16x8& f1, const bf16x8* ip) {
  f32x16 t = MFMA32B(f0, ip[0], zero16());
  return MFMA32B(f1, ip[1], t);
}

constexpr int VJP_SPLIT_MAX_BLOCKS = 256;  // one block (4 waves) per CU, one wave per SIMD

// The Fisher product's reverse half and the policy gradient's VJP (trpo.py:42-43, 58):
// per-wave partials of sum_rows J^T ghead in flat theta layout (one slab row per wave,
// reduced in fixed order by mrl_reduce_rows_f32), from the cached f32 h1 / h2, with the
// split-operand products.  The bf16 mode's transpose-free scheme (mlp_bf16.hip): F tiles
// become T tiles by identity MFMAs -- one per split part, exact, since each part is a
// bf16 value -- and the weight gradients take T tiles as both operands.
template <int SH>
__global__ __launch_bounds__(256, 1) void mlp_vjp_split_kernel(VjpSplitArgs a_in, const float* __restrict__ img_g,
                                                              const int32_t* __restrict__ skip) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const VjpSplitArgs a = vjp_shape_s<SH>(a_in);
  const MlpDims& d = a.d;
  const BDims& b = a.b;
  // the backward parts of the split image: W2 (bw2) and W1^T (bt1) fragments, part p of
  // a segment at (seg - fwd_words) + p BW
  const int BW = split_bw(b), f0 = split_fwd_words(b);
  for (int i = threadIdx.x; i < 3 * BW / 4; i += 256)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g + f0)[i];
  __syncthreads();
  auto wfrag = [&](int seg, int p, int f, int lane) { return frag_at(lds, seg - b.fwd_words + p * BW, f, lane); };
  const int lane = threadIdx.x & 63, h = lane >> 5, j32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile indices
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
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t row = tile * 32 + j32;
    const int64_t rc = row < a.n ? row : 0;
    // validity as opaque 0 / 1 factors (a select on a loaded value becomes a branch and a
    // vmcnt(0) drain); rows past the batch read row 0 and contribute zero head gradients
    float fv = (row < a.n && h == 0) ? 1.f : 0.f, fx = row < a.n ? 1.f : 0.f;
    asm volatile("" : "+v"(fv), "+v"(fx));
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
    f32x16 h1[2], h2[2];
    cache_load(ct, lane, 0, h1[0]);
    cache_load(ct, lane, 1, h1[1]);
    cache_load(ct, lane, 2, h2[0]);
    cache_load(ct, lane, 3, h2[1]);
    const float* gp = a.ghead + rc * a.gh;
    float g8[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      g8[o] = o < A ? gp[o < A ? o : 0] * fv : 0.f;
      gb2[o] += g8[o];
    }
#pragma unroll
    for (int q = 0; q < MAX_OUT; ++q) gls[q] += q < a.n_sum ? gp[A + (q < a.n_sum ? q : 0)] * fv : 0.f;
    float xv[8 * MAX_KS0B];
    const float* xp = a.x + rc * a.n_obs;
#pragma unroll
    for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int k = 16 * s0 + 8 * h + jj;
        xv[8 * s0 + jj] = (s0 < b.KS0B && k < a.n_obs) ? xp[k < a.n_obs ? k : 0] * fx : 0.f;
      }

    // gh2 = W2 . G (F layout, K = head outputs), ga2 = gh2 (1 - h2^2)
    bf16x8 gB[3];
    split8v(g8, gB);
    f32x16 ga2[2];
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) {
      const bf16x8 w[3] = {wfrag(b.bw2, 0, mo, lane), wfrag(b.bw2, 1, mo, lane), wfrag(b.bw2, 2, mo, lane)};
      ga2[mo] = zero16();
      mma_split<MRL_SPLIT_NPROD>(w, gB, ga2[mo]);
      mul_dtanh16(ga2[mo], h2[mo]);
    }
    // gW2 += H2^T G: T parts of G (D[row][o]) and of H2 (D[row][u2])
    {
      bf16x8 gT[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const f32x16 t = MFMA32B(gB[p], ident_nat(0, lane), zero16());
        gT[0][p] = pack8(t, 0);
        gT[1][p] = pack8(t, 1);
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        bf16x8 f0[3], f1[3];
        split8(h2[m], 0, f0);
        split8(h2[m], 1, f1);
        bf16x8 hT[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const f32x16 t = transpose_ff(f0[p], f1[p], ip);
          hT[0][p] = pack8(t, 0);
          hT[1][p] = pack8(t, 1);
        }
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) mma_split<MRL_SPLIT_NPROD>(hT[sp], gT[sp], gW2[m]);
      }
    }
    VJP_SPLIT_FENCE();
    // ga2 as F-fragment parts (A operand of gh1) and T-fragment parts (B operand of gW1)
    bf16x8 gaF[4][3], gaT[2][2][3];  // [s][p], [m][sp][p]
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      split8(ga2[m], 0, gaF[2 * m]);
      split8(ga2[m], 1, gaF[2 * m + 1]);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const f32x16 t = transpose_ff(gaF[2 * m][p], gaF[2 * m + 1][p], ip);
#pragma unroll
        for (int r = 0; r < 16; ++r) gb1[m] += t[r];
        gaT[m][0][p] = pack8(t, 0);
        gaT[m][1][p] = pack8(t, 1);
      }
    }
    // the inputs in T layout (D[row][in]), per part
    bf16x8 xT[2][3];
    {
      bf16x8 xs[MAX_KS0B][3];
#pragma unroll
      for (int s0 = 0; s0 < MAX_KS0B; ++s0) split8v(xv + 8 * s0, xs[s0]);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        f32x16 t = zero16();
#pragma unroll
        for (int s0 = 0; s0 < MAX_KS0B; ++s0)
          if (s0 < b.KS0B) t = MFMA32B(xs[s0][p], ident_nat(16 * s0, lane), t);
        xT[0][p] = pack8(t, 0);
        xT[1][p] = pack8(t, 1);
      }
    }
    VJP_SPLIT_FENCE();
    // per u1 tile: gh1 (T layout) = ga2 . W1^T, ga1 = gh1 (1 - h1^2), then
    // gW1 += H1^T GA2 and gW0 += X^T GA1
#pragma unroll
    for (int no = 0; no < 2; ++no) {
      f32x16 ga1 = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 w[3] = {wfrag(b.bt1, 0, no * 4 + s, lane), wfrag(b.bt1, 1, no * 4 + s, lane),
                             wfrag(b.bt1, 2, no * 4 + s, lane)};
        mma_split<MRL_SPLIT_NPROD>(gaF[s], w, ga1);
      }
      bf16x8 f0[3], f1[3];
      split8(h1[no], 0, f0);
      split8(h1[no], 1, f1);
      bf16x8 hT[2][3];
      f32x16 h1T = zero16();
#pragma unroll
      for (int p = 2; p >= 0; --p) {  // h1 = (lo + mid) + hi: exact, the parts reassemble the f32 value
        const f32x16 t = transpose_ff(f0[p], f1[p], ip);
        h1T += t;
        hT[0][p] = pack8(t, 0);
        hT[1][p] = pack8(t, 1);
      }
      mul_dtanh16(ga1, h1T);
#pragma unroll
      for (int r = 0; r < 16; ++r) gb0[no] += ga1[r];
      bf16x8 g1[2][3];
      split8(ga1, 0, g1[0]);
      split8(ga1, 1, g1[1]);
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        mma_split<MRL_SPLIT_NPROD>(hT[sp], gaT[0][sp], gW1[no][0]);
        mma_split<MRL_SPLIT_NPROD>(hT[sp], gaT[1][sp], gW1[no][1]);
        mma_split<MRL_SPLIT_NPROD>(xT[sp], g1[sp], gW0[no]);
      }
      VJP_SPLIT_FENCE();
    }
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


// ---- VJP, second form: no identity transposes.  The T-layout operands come straight
// from memory (h1 / h2 gathered from the f32 cache in T order -- the tile was just
// streamed, the gathers hit L2 --, the inputs and head rows from their row arrays) and
// ga2 is formed in both layouts by MFMA (K = head outputs, one k-step): gh2_F = W2 . G
// for gh1 and gh2_T = G . W2^T for gW1.  168 part MFMAs per 32-row tile instead of 198.
// element (row j, unit w of 32-unit slot `slot`) of an f32 cache tile
__device__ inline int cache_off_s(int slot, int j, int w) {
  return ((slot * 4 + (w >> 3)) * 64 + 32 * ((w >> 2) & 1) + j) * 4 + (w & 3);
}

// T-order row r of a 32-row tile relative to lane half hq's first row: cperm(r, hq) - 4 hq
__device__ constexpr int trow_c(int r) { return (r & 3) + 8 * (r >> 2); }
// lane part of the T-order cache gathers (cache_off_s minus the slot and row constants):
// element (slot, cperm(r, hq), cq) sits at this + slot * 1024 + 4 trow_c(r), so every
// gather is one base register plus an immediate offset
__device__ inline int cache_lane_off(int hq, int cq) {
  return ((cq >> 3) * 64 + 32 * ((cq >> 2) & 1)) * 4 + (cq & 3) + 16 * hq;
}
// a T-order row gather of a [rows][w] f32 array (inputs, head rows): column col of the
// tile's row cperm(r, hq); rows past n read as 0 (full tiles take the immediate-offset
// path, the batch's last tile the clamped one)
template <int NR>
__device__ inline void trow_gather(const float* base, int64_t w, int64_t row0, int hq, int col, bool col_ok, int64_t n,
                                   float* out) {
  const float fc = col_ok ? 1.f : 0.f;
  const int cc = col_ok ? col : 0;
  if (row0 + 32 <= n) {
    const float* p = base + (row0 + 4 * hq) * w + cc;
#pragma unroll
    for (int r = 0; r < NR; ++r) out[r] = p[trow_c(r) * w] * fc;
  } else {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t rw = row0 + 4 * hq + trow_c(r);
      float f = rw < n ? fc : 0.f;
      asm volatile("" : "+v"(f));
      out[r] = base[(rw < n ? rw : 0) * w + cc] * f;
    }
  }
}

template <int SH>
__global__ __launch_bounds__(256, 1) void mlp_vjp_split2_kernel(VjpSplitArgs a_in, const float* __restrict__ img_g,
                                                               const int32_t* __restrict__ skip) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const VjpSplitArgs a = vjp_shape_s<SH>(a_in);
  const MlpDims& d = a.d;
  const BDims& b = a.b;
  const int BW = split_bw(b), f0 = split_fwd_words(b);
  for (int i = threadIdx.x; i < 3 * BW / 4; i += 256)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g + f0)[i];
  __syncthreads();
  auto wfrag = [&](int seg, int p, int f, int lane) { return frag_at(lds, seg - b.fwd_words + p * BW, f, lane); };
  const int lane = threadIdx.x & 63, h = lane >> 5, j32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile indices
  const int A = d.A;
  f32x16 gW2[2], gW1[2][2], gW0[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    gW2[m] = zero16();
    gW0[m] = zero16();
#pragma unroll
    for (int n = 0; n < 2; ++n) gW1[m][n] = zero16();
  }
  float gb0[2] = {0.f, 0.f}, gb1[2] = {0.f, 0.f};
  float gb2[MAX_OUT], gls[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    gb2[o] = 0.f;
    gls[o] = 0.f;
  }
  // T-layout lane roles: column c = lane & 31 (a unit, an input or a head output), register
  // r of lane half h holds row cperm(r, h) of the tile
  const int c = j32;
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t row0 = tile * 32, row = row0 + j32;
    const int64_t rc = row < a.n ? row : 0;
    float fv = (row < a.n && h == 0) ? 1.f : 0.f;
    asm volatile("" : "+v"(fv));
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
    int hq = h, cq = c;  // opaque lane coordinates (see mlp_fisher_split_kernel)
    asm volatile("" : "+v"(hq), "+v"(cq));
    // F-layout h2 (tanh' of gh2_F); the T-layout operands are gathered phase by phase
    f32x16 h2F[2];
    cache_load(ct, lane, 2, h2F[0]);
    cache_load(ct, lane, 3, h2F[1]);
    // row of register r in a T tile, and its validity factor
    const float* cb = ct + cache_lane_off(hq, cq);
    auto gather_cache = [&](int slot, f32x16& t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = cb[slot * 1024 + 4 * trow_c(r)];
    };
    const float* gp = a.ghead + rc * a.gh;
    float g8[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      g8[o] = o < A ? gp[o < A ? o : 0] * fv : 0.f;
      gb2[o] += g8[o];
    }
#pragma unroll
    for (int q = 0; q < MAX_OUT; ++q) gls[q] += q < a.n_sum ? gp[A + (q < a.n_sum ? q : 0)] * fv : 0.f;

    bf16x8 gB[3];
    split8v(g8, gB);
    bf16x8 gs[2][3];  // G in T layout (D[row][o])
    {
      f32x16 gT;
float gv[16];
      trow_gather<16>(a.ghead, a.gh, row0, hq, cq, c < A, a.n, gv);
#pragma unroll
      for (int r = 0; r < 16; ++r) gT[r] = gv[r];
      split8(gT, 0, gs[0]);
      split8(gT, 1, gs[1]);
    }
    // ga2 in both layouts (gb1 from the T one); gW2 += H2^T G
    bf16x8 gaF[4][3], gaT[2][2][3];
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) {
      f32x16 h2T;
      gather_cache(2 + mo, h2T);
      const bf16x8 w[3] = {wfrag(b.bw2, 0, mo, lane), wfrag(b.bw2, 1, mo, lane), wfrag(b.bw2, 2, mo, lane)};
      f32x16 gf = zero16(), gt = zero16();
      mma_split<MRL_SPLIT_NPROD>(w, gB, gf);   // D[u2][row]
      mma_split<MRL_SPLIT_NPROD>(gB, w, gt);   // D[row][u2]
      mul_dtanh16(gf, h2F[mo]);
      mul_dtanh16(gt, h2T);
#pragma unroll
      for (int r = 0; r < 16; ++r) gb1[mo] += gt[r];
      split8(gf, 0, gaF[2 * mo]);
      split8(gf, 1, gaF[2 * mo + 1]);
      split8(gt, 0, gaT[mo][0]);
      split8(gt, 1, gaT[mo][1]);
      bf16x8 hs[2][3];
      split8(h2T, 0, hs[0]);
      split8(h2T, 1, hs[1]);
      mma_split<MRL_SPLIT_NPROD>(hs[0], gs[0], gW2[mo]);
      mma_split<MRL_SPLIT_NPROD>(hs[1], gs[1], gW2[mo]);
    }
    bf16x8 xs[2][3];
    {
      f32x16 xT;
float xv[16];
      trow_gather<16>(a.x, a.n_obs, row0, hq, cq, c < a.n_obs, a.n, xv);
#pragma unroll
      for (int r = 0; r < 16; ++r) xT[r] = xv[r];
      split8(xT, 0, xs[0]);
      split8(xT, 1, xs[1]);
    }
#pragma unroll
    for (int no = 0; no < 2; ++no) {
      f32x16 h1T;
      gather_cache(no, h1T);
      f32x16 ga1 = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 w[3] = {wfrag(b.bt1, 0, no * 4 + s, lane), wfrag(b.bt1, 1, no * 4 + s, lane),
                             wfrag(b.bt1, 2, no * 4 + s, lane)};
        mma_split<MRL_SPLIT_NPROD>(gaF[s], w, ga1);
      }
      mul_dtanh16(ga1, h1T);
#pragma unroll
      for (int r = 0; r < 16; ++r) gb0[no] += ga1[r];
      bf16x8 hs[2][3], g1[2][3];
      split8(h1T, 0, hs[0]);
      split8(h1T, 1, hs[1]);
      split8(ga1, 0, g1[0]);
      split8(ga1, 1, g1[1]);
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        mma_split<MRL_SPLIT_NPROD>(hs[sp], gaT[0][sp], gW1[no][0]);
        mma_split<MRL_SPLIT_NPROD>(hs[sp], gaT[1][sp], gW1[no][1]);
        mma_split<MRL_SPLIT_NPROD>(xs[sp], g1[sp], gW0[no]);
      }
    }
  }
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


// An LDS pointer the compiler cannot see through: accesses at constant offsets from it
// fold into the ds instructions' 16-bit offset field.  LDS data past 64 KB addressed from
// the segment base instead needs one address register per fragment, which the compiler
// hoists out of the row loop -- dozens of loop-invariant registers, spilled.
__device__ inline const float* lds_opaque(const float* p) {
  auto q = (const __attribute__((address_space(3))) float*)p;
  asm volatile("" : "+v"(q));
  return (const float*)q;
}

// ---- the whole Fisher product in one pass (trpo.py:45-58, 86-92): per 32-row tile the
// JVP of mlp_fvp_split_kernel, the KL-metric head rows (fvp_metric_row) kept in
// registers, then the VJP of mlp_vjp_split2_kernel on them -- the activation cache is
// read once (h1 / h2 streamed in F order; the T-order gathers of the VJP hit the lines
// just streamed) and the head rows never go to memory.  The G tile in T order (B operand
// of gW2 += H2^T G) comes through a 1 KB LDS tile per wave instead of a global gather.
// Grid and tile order are the VJP's (one slab row per wave, the same tiles per wave), so
// the slab -- and the Fisher product -- is bit-identical to the two-pass split path
// (split JVP rows, then mlp_vjp_split2_kernel on the rows it wrote).
template <int SH>
__global__ __launch_bounds__(256, 1) void mlp_fisher_split_kernel(RowsArgs a, BDims b, float* __restrict__ slab,
                                                                 const float* __restrict__ img_g,
                                                                 const float* __restrict__ imt_g,
                                                                 const int32_t* __restrict__ skip) {
  split_shape<SH>(a, b);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  // LDS: the primal split image whole (forward + backward parts), the tangent's forward
  // parts, then one 32 x 8 head-row tile per wave
  const int WP = split_image_words(b), WT = split_fwd_words(b), PS = split_fw(b), BW = split_bw(b);
  for (int i = threadIdx.x; i < WP / 4; i += 256)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
  for (int i = threadIdx.x; i < WT / 4; i += 256)
    reinterpret_cast<float4*>(lds + WP)[i] = reinterpret_cast<const float4*>(imt_g)[i];
  __syncthreads();
  const float* img = lds;
  const float* imt = lds_opaque(lds + WP);  // the tangent image lies past 64 KB
  const int lane = threadIdx.x & 63, h = lane >> 5, j32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile indices
  float* gtile = lds + WP + WT + wave * 256;
  auto wfrag = [&](int seg, int p, int f) { return frag_at(lds, WT + seg - b.fwd_words + p * BW, f, lane); };
  const MlpDims dd = head_dims(a.d, b);
  const MlpDims& d = a.d;
  const int A = a.A;
  const int n_sum = a.head == MRL_HEAD_GAUSS ? A : 0;
  float ls[MAX_OUT], sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
  for (int j = 0; j < MAX_OUT; ++j) {
    ls[j] = (a.logstd != nullptr && j < A) ? a.logstd[j] : 0.f;
    sd[j] = expf(ls[j]);
    dls[j] = (a.dlogstd != nullptr && j < A) ? a.dlogstd[j] : 0.f;
  }
  const bool need_z = a.head != MRL_HEAD_GAUSS;
  f32x16 gW2[2], gW1[2][2], gW0[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    gW2[m] = zero16();
    gW0[m] = zero16();
#pragma unroll
    for (int n = 0; n < 2; ++n) gW1[m][n] = zero16();
  }
  float gb0[2] = {0.f, 0.f}, gb1[2] = {0.f, 0.f};
  float gb2[MAX_OUT], gls[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    gb2[o] = 0.f;
    gls[o] = 0.f;
  }
  const int c = j32;
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t row0 = tile * 32, row = row0 + j32;
    const bool valid = row < a.n;
    float fv = (valid && h == 0) ? 1.f : 0.f, fx = valid ? 1.f : 0.f;
    asm volatile("" : "+v"(fv), "+v"(fx));
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
    XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, row, valid};
    // per-lane T-order indices from opaque copies of the lane coordinates: derived anew
    // each tile next to their use, not hoisted out of the loop as ~50 live registers
    int hq = h, cq = c;
    asm volatile("" : "+v"(hq), "+v"(cq));
    // ---- JVP (mlp_fvp_split_kernel): dh = (x dW0 + db0) (1 - h1^2), then per output
    // tile da = (dh W1 + h1 dW1 + db1) (1 - h2^2) and the head on the f32 VALU
    f32x16 h2F[2];
    float z[MAX_OUT], dz[MAX_OUT];
    {
      f32x16 h1[2], dh[2];
      cache_load(ct, lane, 0, h1[0]);
      cache_load(ct, lane, 1, h1[1]);
      dh[0] = load_bias16(imt, b.fb0, 0, h);
      dh[1] = load_bias16(imt, b.fb0, 1, h);
#pragma unroll
      for (int s0 = 0; s0 < MAX_KS0B; ++s0) {
        if (s0 < b.KS0B) {
          float xv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = xl(16 * s0 + 8 * h + j);
          bf16x8 xs[3];
          split8v(xv, xs);
          mfma_split<MRL_SPLIT_NPROD>(imt, b.fa0, PS, 0 * b.KS0B + s0, lane, xs, dh[0]);
          mfma_split<MRL_SPLIT_NPROD>(imt, b.fa0, PS, 1 * b.KS0B + s0, lane, xs, dh[1]);
        }
      }
      mul_dtanh16(dh[0], h1[0]);
      mul_dtanh16(dh[1], h1[1]);
      float dzt[MAX_OUT];
#pragma unroll
      for (int o = 0; o < MAX_OUT; ++o) z[o] = dz[o] = dzt[o] = 0.f;
      f32x16 da2[2] = {load_bias16(imt, b.fb1, 0, h), load_bias16(imt, b.fb1, 1, h)};
#pragma unroll
      for (int s = 0; s < 4; ++s) {  // each input fragment split once (mlp_fvp_split_kernel)
        bf16x8 ps[3];
        split8(dh[s >> 1], s & 1, ps);
        mfma_split<MRL_SPLIT_NPROD>(img, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
        mfma_split<MRL_SPLIT_NPROD>(img, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
      }
      FVP_SPLIT_FENCE();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 ps[3];
        split8(h1[s >> 1], s & 1, ps);
        mfma_split<MRL_SPLIT_NPROD>(imt, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
        mfma_split<MRL_SPLIT_NPROD>(imt, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
      }
      FVP_SPLIT_FENCE();
#pragma unroll
      for (int mo = 0; mo < 2; ++mo) {
        f32x16& da = da2[mo];
        cache_load(ct, lane, 2 + mo, h2F[mo]);
        mul_dtanh16(da, h2F[mo]);
        if (need_z) head_partial_mt(img, dd, h2F[mo], mo, h, z);
        head_partial_mt(img, dd, da, mo, h, dz);
        head_partial_mt(imt, dd, h2F[mo], mo, h, dzt);
        FVP_SPLIT_FENCE();
      }
      if (need_z) head_finish(img, dd, z);
#pragma unroll
      for (int o = 0; o < MAX_OUT; ++o) dz[o] += dzt[o];
      head_finish(imt, dd, dz);
    }
    FVP_SPLIT_FENCE();
    // ---- the metric's head rows (every lane forms its row's; lane half 0 owns them)
    static_assert(MAX_OUT == 8, "the head-row tile holds 8 columns");
    float gm[MAX_OUT], gl[MAX_OUT];
    fvp_metric_row<MAX_OUT>(a, z, dz, sd, dls, gm, gl);
    float g8[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      g8[o] = o < A ? gm[o] * fv : 0.f;
      gb2[o] += g8[o];
    }
#pragma unroll
    for (int q = 0; q < MAX_OUT; ++q) gls[q] += q < n_sum ? gl[q] * fv : 0.f;
    // G in T order through the wave's LDS tile: row j32's values from lane half 0
    if (h == 0) {
      reinterpret_cast<float4*>(gtile + 8 * j32)[0] = make_float4(gm[0], gm[1], gm[2], gm[3]);
      reinterpret_cast<float4*>(gtile + 8 * j32)[1] = make_float4(gm[4], gm[5], gm[6], gm[7]);
    }
    WAVE_LDS_ORDER();
    bf16x8 gs[2][3];
    {
      f32x16 gT;
      const float* gb = gtile + 32 * hq + (cq & 7);
      const float fc = c < A ? 1.f : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float f = row0 + 4 * hq + trow_c(r) < a.n ? fc : 0.f;
        asm volatile("" : "+v"(f));
        gT[r] = gb[8 * trow_c(r)] * f;
      }
      split8(gT, 0, gs[0]);
      split8(gT, 1, gs[1]);
    }
    WAVE_LDS_ORDER();  // the next tile's writes stay behind these reads
    VJP_SPLIT_FENCE();
    // ---- VJP (mlp_vjp_split2_kernel) of the head rows
    const float* cb = ct + cache_lane_off(hq, cq);
    auto gather_cache = [&](int slot, f32x16& t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = cb[slot * 1024 + 4 * trow_c(r)];
    };
    bf16x8 gB[3];
    split8v(g8, gB);
    bf16x8 gaF[4][3], gaT[2][2][3];
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) {
      f32x16 h2T;
      gather_cache(2 + mo, h2T);
      const bf16x8 w[3] = {wfrag(b.bw2, 0, mo), wfrag(b.bw2, 1, mo), wfrag(b.bw2, 2, mo)};
      f32x16 gf = zero16(), gt = zero16();
      mma_split<MRL_SPLIT_NPROD>(w, gB, gf);
      mma_split<MRL_SPLIT_NPROD>(gB, w, gt);
      mul_dtanh16(gf, h2F[mo]);
      mul_dtanh16(gt, h2T);
#pragma unroll
      for (int r = 0; r < 16; ++r) gb1[mo] += gt[r];
      split8(gf, 0, gaF[2 * mo]);
      split8(gf, 1, gaF[2 * mo + 1]);
      split8(gt, 0, gaT[mo][0]);
      split8(gt, 1, gaT[mo][1]);
      bf16x8 hs[2][3];
      split8(h2T, 0, hs[0]);
      split8(h2T, 1, hs[1]);
      mma_split<MRL_SPLIT_NPROD>(hs[0], gs[0], gW2[mo]);
      mma_split<MRL_SPLIT_NPROD>(hs[1], gs[1], gW2[mo]);
      VJP_SPLIT_FENCE();
    }
    bf16x8 xs[2][3];
    {
      f32x16 xT;
float xv[16];
      trow_gather<16>(a.x, a.n_obs, row0, hq, cq, c < a.n_obs, a.n, xv);
#pragma unroll
      for (int r = 0; r < 16; ++r) xT[r] = xv[r];
      split8(xT, 0, xs[0]);
      split8(xT, 1, xs[1]);
    }
#pragma unroll
    for (int no = 0; no < 2; ++no) {
      f32x16 h1T;
      gather_cache(no, h1T);
      f32x16 ga1 = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 w[3] = {wfrag(b.bt1, 0, no * 4 + s), wfrag(b.bt1, 1, no * 4 + s), wfrag(b.bt1, 2, no * 4 + s)};
        mma_split<MRL_SPLIT_NPROD>(gaF[s], w, ga1);
      }
      mul_dtanh16(ga1, h1T);
#pragma unroll
      for (int r = 0; r < 16; ++r) gb0[no] += ga1[r];
      bf16x8 hs[2][3], g1[2][3];
      split8(h1T, 0, hs[0]);
      split8(h1T, 1, hs[1]);
      split8(ga1, 0, g1[0]);
      split8(ga1, 1, g1[1]);
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        mma_split<MRL_SPLIT_NPROD>(hs[sp], gaT[0][sp], gW1[no][0]);
        mma_split<MRL_SPLIT_NPROD>(hs[sp], gaT[1][sp], gW1[no][1]);
        mma_split<MRL_SPLIT_NPROD>(xs[sp], g1[sp], gW0[no]);
      }
      VJP_SPLIT_FENCE();
    }
    if (a.ghead != nullptr && valid && h == 0) {  // diagnostic: the head rows as the two-pass path writes them
#pragma unroll
      for (int j = 0; j < MAX_OUT; ++j) {
        if (j < A) {
          a.ghead[row * a.gh + j] = gm[j];
          if (a.head == MRL_HEAD_GAUSS) a.ghead[row * a.gh + A + j] = gl[j];
        }
      }
    }
  }
  float* out = slab + ((int64_t)blockIdx.x * 4 + wave) * d.P;
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
  for (int q = 0; q < n_sum; ++q) {
    const float sum = wave_sumf(gls[q]);
    if (lane == 0) out[d.tls + q] = sum;
  }
}

}  // namespace mrl

using namespace mrl;

static int check_desc_s(const mrl_mlp_desc* d) {
  if (d == nullptr) return fail(E_ARG, "null mlp desc");
  if (d->n_hidden != HID || d->n_layers != 2)
    return fail(E_UNSUPPORTED, "only hid_sizes=[64,64] is implemented on the fused HIP path");
  if (d->n_in < 1 || d->n_in > MAX_IN) return fail(E_UNSUPPORTED, "n_in must be in [1, 32]");
  if (d->n_out < 1 || d->n_out > MAX_OUT) return fail(E_UNSUPPORTED, "n_out must be in [1, 8]");
  if (d->head < 0 || d->head > 2) return fail(E_ARG, "bad head kind");
  if (d->head == MRL_HEAD_LINEAR && d->n_out != 1) return fail(E_ARG, "linear head needs n_out=1");
  return OK;
}

static int static_shape_split(const mrl_mlp_desc* d) {
#ifdef MRL_NO_STATIC_SHAPES
  (void)d;
  return 0;
#else
  for (int i = 1; i < N_STATIC_SHAPES; ++i)
    if (STATIC_SHAPES[i].O == d->n_in && STATIC_SHAPES[i].A == d->n_out && STATIC_SHAPES[i].head == d->head) return i;
  return 0;
#endif
}

// grid: two resident rounds (MRL_SPLIT_BLOCKS overrides)
static int64_t split_rows_blocks(int64_t n) {
  static const int64_t env_cap = [] {
    const char* e = getenv("MRL_SPLIT_BLOCKS");
    return (int64_t)(e ? atoi(e) : 0);
  }();
  // two resident rounds: 256 CUs x (4 waves per SIMD worth of blocks)
  const int64_t cap = env_cap > 0 ? env_cap : 2 * 256 * (4 * MRL_SPLIT_FVP_OCC / SPLIT_ROWS_WAVES > 0
                                                         ? 4 * MRL_SPLIT_FVP_OCC / SPLIT_ROWS_WAVES : 1);
  int64_t g = ((n + 31) / 32 + SPLIT_ROWS_WAVES - 1) / SPLIT_ROWS_WAVES;
  if (g < 1) g = 1;
  return g > cap ? cap : g;
}

extern "C" {

int64_t mrl_mlp_image_words_split(const mrl_mlp_desc* d) {
  if (check_desc_s(d) != OK) return -1;
  return split_image_words(bf16_dims(d->n_in, d->n_out));
}

int mrl_mlp_pack_split(const mrl_mlp_desc* d, const float* theta, float* image, int32_t fwd_only, const int32_t* skip,
                       void* stream) {
  int rc = check_desc_s(d);
  if (rc) return rc;
  if (!theta || !image) return fail(E_ARG, "null pointer");
  const MlpDims m = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  const BDims b = bf16_dims(d->n_in, d->n_out);
  const int words = fwd_only ? split_fwd_words(b) : split_image_words(b);
  hipLaunchKernelGGL(mlp_pack_split_kernel, dim3((words + 255) / 256), dim3(256), 0, (hipStream_t)stream, m, b, theta,
                     image, words, skip);
  return hip_check(hipGetLastError(), "mrl_mlp_pack_split");
}

int mrl_mlp_fvp_split(const mrl_mlp_desc* d, const float* theta, const float* image, const float* tangent,
                      const float* image_t, const mrl_rows_io* io, const int32_t* skip, void* stream) {
  int rc = check_desc_s(d);
  if (rc) return rc;
  if (!io || !image || !image_t || !tangent || !io->x || !io->ghead) return fail(E_ARG, "null pointer");
  if (!io->act_cache || io->cache_mode != MRL_CACHE_READ)
    return fail(E_ARG, "mrl_mlp_fvp_split reads the f32 activation cache (MRL_CACHE_READ)");
  if (io->ep_t) return fail(E_ARG, "mrl_mlp_fvp_split: policy rows only (no time feature)");
  if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "Fisher product of a value net");
  if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
  if (io->n <= 0) return OK;
  RowsArgs a{};
  a.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  a.head = d->head;
  a.n_obs = d->n_in;
  a.gh = d->head == MRL_HEAD_GAUSS ? 2 * d->n_out : d->n_out;
  a.A = d->n_out;
  a.x = io->x;
  a.n = io->n;
  a.inv_ng = io->inv_n_global;
  a.ghead = io->ghead;
  a.logstd = (d->head == MRL_HEAD_GAUSS && theta) ? theta + a.d.tls : nullptr;
  a.dlogstd = (d->head == MRL_HEAD_GAUSS && tangent) ? tangent + a.d.tls : nullptr;
  a.cache = io->act_cache;
  a.cache_mode = MRL_CACHE_READ;
  const BDims b = bf16_dims(d->n_in, d->n_out);
  const size_t shm = (size_t)split_fwd_words(b) * 4 * 2;
  const dim3 grid(split_rows_blocks(io->n)), blk(SPLIT_ROWS_BLOCK);
  hipStream_t s = (hipStream_t)stream;
  switch (static_shape_split(d)) {
    case 1: hipLaunchKernelGGL((mlp_fvp_split_kernel<1>), grid, blk, shm, s, a, b, image, image_t, skip); break;
    case 2: hipLaunchKernelGGL((mlp_fvp_split_kernel<2>), grid, blk, shm, s, a, b, image, image_t, skip); break;
    default: hipLaunchKernelGGL((mlp_fvp_split_kernel<0>), grid, blk, shm, s, a, b, image, image_t, skip); break;
  }
  return hip_check(hipGetLastError(), "mrl_mlp_fvp_split");
}

int mrl_mlp_vjp_split(const mrl_mlp_desc* d, const float* image, const float* x, const float* ghead, int64_t n,
                      float* slab, const float* act_cache, const int32_t* skip, void* stream) {
  int rc = check_desc_s(d);
  if (rc) return rc;
  if (!image || !x || !ghead || !slab || !act_cache) return fail(E_ARG, "null pointer");
  if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "mrl_mlp_vjp_split: policy nets only");
  if (n <= 0) return OK;
  VjpSplitArgs a{};
  a.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  a.b = bf16_dims(d->n_in, d->n_out);
  a.n_obs = d->n_in;
  a.n_sum = d->head == MRL_HEAD_GAUSS ? d->n_out : 0;
  a.gh = d->n_out + a.n_sum;
  a.x = x;
  a.n = n;
  a.ghead = ghead;
  a.slab = slab;
  a.cache = act_cache;
  // the slab rows of mrl_mlp_slab_rows(d, n): one row per wave of a 4-wave block
  const int64_t cus = d->cus > 0 ? d->cus : 256;
  int64_t blocks = ((n + 31) / 32 + 3) / 4;
  const int64_t cap = VJP_SPLIT_MAX_BLOCKS * cus / 256 > 0 ? VJP_SPLIT_MAX_BLOCKS * cus / 256 : 1;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  const size_t shm = (size_t)3 * split_bw(a.b) * 4;
  const dim3 grid(blocks), blk(256);
  hipStream_t s = (hipStream_t)stream;
  // MRL_VJP_SPLIT_FORM=2: the transpose-free second form (read per call: tests switch it)
  const char* fe = getenv("MRL_VJP_SPLIT_FORM");
  const int form = fe ? atoi(fe) : 1;
  const int sh = static_shape_split(d);
  if (form == 2) {
    if (sh == 1) hipLaunchKernelGGL((mlp_vjp_split2_kernel<1>), grid, blk, shm, s, a, image, skip);
    else if (sh == 2) hipLaunchKernelGGL((mlp_vjp_split2_kernel<2>), grid, blk, shm, s, a, image, skip);
    else hipLaunchKernelGGL((mlp_vjp_split2_kernel<0>), grid, blk, shm, s, a, image, skip);
  } else {
    if (sh == 1) hipLaunchKernelGGL((mlp_vjp_split_kernel<1>), grid, blk, shm, s, a, image, skip);
    else if (sh == 2) hipLaunchKernelGGL((mlp_vjp_split_kernel<2>), grid, blk, shm, s, a, image, skip);
    else hipLaunchKernelGGL((mlp_vjp_split_kernel<0>), grid, blk, shm, s, a, image, skip);
  }
  return hip_check(hipGetLastError(), "mrl_mlp_vjp_split");
}

int mrl_mlp_fisher_split(const mrl_mlp_desc* d, const float* theta, const float* image, const float* tangent,
                         const float* image_t, const mrl_rows_io* io, float* slab, const int32_t* skip,
                         void* stream) {
  int rc = check_desc_s(d);
  if (rc) return rc;
  if (!io || !image || !image_t || !tangent || !io->x || !slab) return fail(E_ARG, "null pointer");
  if (!io->act_cache || io->cache_mode != MRL_CACHE_READ)
    return fail(E_ARG, "mrl_mlp_fisher_split reads the f32 activation cache (MRL_CACHE_READ)");
  if (io->ep_t) return fail(E_ARG, "mrl_mlp_fisher_split: policy rows only (no time feature)");
  if (d->head == MRL_HEAD_LINEAR) return fail(E_ARG, "Fisher product of a value net");
  if (d->head == MRL_HEAD_GAUSS && !theta) return fail(E_ARG, "DiagGauss needs theta (logstd)");
  if (io->n <= 0) return OK;
  RowsArgs a{};
  a.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  a.head = d->head;
  a.n_obs = d->n_in;
  a.gh = d->head == MRL_HEAD_GAUSS ? 2 * d->n_out : d->n_out;
  a.A = d->n_out;
  a.x = io->x;
  a.n = io->n;
  a.inv_ng = io->inv_n_global;
  a.ghead = io->ghead;  // optional: the head rows, as the two-pass path writes them
  a.logstd = (d->head == MRL_HEAD_GAUSS && theta) ? theta + a.d.tls : nullptr;
  a.dlogstd = (d->head == MRL_HEAD_GAUSS && tangent) ? tangent + a.d.tls : nullptr;
  a.cache = io->act_cache;
  a.cache_mode = MRL_CACHE_READ;
  const BDims b = bf16_dims(d->n_in, d->n_out);
  // the VJP's grid (mrl_mlp_slab_rows): one slab row per wave of a 4-wave block
  const int64_t cus = d->cus > 0 ? d->cus : 256;
  int64_t blocks = ((io->n + 31) / 32 + 3) / 4;
  const int64_t cap = VJP_SPLIT_MAX_BLOCKS * cus / 256 > 0 ? VJP_SPLIT_MAX_BLOCKS * cus / 256 : 1;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  const size_t shm = ((size_t)split_image_words(b) + split_fwd_words(b) + 4 * 256) * 4;
  if (shm > 160 * 1024) return fail(E_UNSUPPORTED, "mrl_mlp_fisher_split: images exceed LDS");
  const dim3 grid(blocks), blk(256);
  hipStream_t s = (hipStream_t)stream;
  switch (static_shape_split(d)) {
    case 1: hipLaunchKernelGGL((mlp_fisher_split_kernel<1>), grid, blk, shm, s, a, b, slab, image, image_t, skip); break;
    case 2: hipLaunchKernelGGL((mlp_fisher_split_kernel<2>), grid, blk, shm, s, a, b, slab, image, image_t, skip); break;
    default: hipLaunchKernelGGL((mlp_fisher_split_kernel<0>), grid, blk, shm, s, a, b, slab, image, image_t, skip); break;
  }
  return hip_check(hipGetLastError(), "mrl_mlp_fisher_split");
}

}  // extern "C"
