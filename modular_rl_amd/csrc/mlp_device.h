// Device building blocks shared by the MLP kernels and the rollout kernel:
// LDS fragment reads, the MFMA layer chains of the transposed-activation layout
// (see mlp_layout.h) and small wave utilities.
#pragma once
#include "mlp_layout.h"

// Cross-lane hand-off through LDS inside ONE wave: a wave's LDS instructions execute
// in issue order, so only the compiler must be kept from moving loads above stores.
#define WAVE_LDS_ORDER() asm volatile("" ::: "memory")

namespace mrl {

// ------------------------------------------------------------------ device helpers
__device__ inline f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ inline float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ inline float f4get(const float4& v, int q) { return q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w)); }

__device__ inline f32x16 load_bias16(const float* lds, int off, int mo, int h) {
  const float* p = lds + off + (mo * 2 + h) * 16;
  const float4 a = ld4(p), b = ld4(p + 4), c = ld4(p + 8), e = ld4(p + 12);
  f32x16 r;
  r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
  r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  r[8] = c.x; r[9] = c.y; r[10] = c.z; r[11] = c.w;
  r[12] = e.x; r[13] = e.y; r[14] = e.z; r[15] = e.w;
  return r;
}

__device__ inline float4 frag4(const float* lds, int seg, int KSp, int mo, int s4, int lane) {
  return reinterpret_cast<const float4*>(lds + seg)[(mo * (KSp / 4) + s4) * 64 + lane];
}

// input-layer operand loader from global memory: x[row, k] (k < n_obs), then the
// VF time feature t / timestep_limit (core.py:659-660) at k == n_obs.
struct XGlobal {
  const float* x;
  const int32_t* ept;
  double ts_limit;
  int n_obs;
  int64_t row;
  bool valid;
  // branch-free: rows past the batch read row 0 and are zeroed at the end
  __device__ inline float operator()(int k) const {
    const int64_t r = valid ? row : 0;
    float v = 0.f;
    if (k < n_obs) v = x[r * n_obs + k];
    else if (ept != nullptr && k == n_obs) v = (float)((double)ept[r] / ts_limit);
    return valid ? v : 0.f;
  }
};

// XGlobal with branch-free column reads (the bf16 kernels): columns past n_obs read the
// last one and, like rows past the batch, are zeroed by an opaque 0 / 1 factor -- k
// depends on the lane, and a select on the loaded value became a branch around the load
// and a vmcnt(0) drain per column.  (The fp32 row kernels keep XGlobal: this form spilled
// there.)
struct XGlobalNB {
  const float* x;
  const int32_t* ept;
  double ts_limit;
  int n_obs;
  int64_t row;
  bool valid;
  __device__ inline float operator()(int k) const {
    const int64_t r = valid ? row : 0;
    float f = (valid && k < n_obs) ? 1.f : 0.f;
    asm volatile("" : "+v"(f));
    float v = x[r * n_obs + (k < n_obs ? k : n_obs - 1)] * f;
    if (ept != nullptr && k == n_obs) v = valid ? (float)((double)ept[r] / ts_limit) : 0.f;
    return v;
  }
};

template <class XL>
__device__ inline void layer0(const float* lds, const MlpDims& d, const XL& xl, int lane, f32x16* acc) {
  const int h = lane >> 5;
  for (int s4 = 0; s4 < d.KS0p / 4; ++s4) {
    const float4 w0 = frag4(lds, d.fa0, d.KS0p, 0, s4, lane);
    const float4 w1 = frag4(lds, d.fa0, d.KS0p, 1, s4, lane);
    const float b0 = xl(8 * s4 + 0 + h), b1 = xl(8 * s4 + 2 + h);
    const float b2 = xl(8 * s4 + 4 + h), b3 = xl(8 * s4 + 6 + h);
    acc[0] = MFMA32(w0.x, b0, acc[0]);
    acc[1] = MFMA32(w1.x, b0, acc[1]);
    acc[0] = MFMA32(w0.y, b1, acc[0]);
    acc[1] = MFMA32(w1.y, b1, acc[1]);
    acc[0] = MFMA32(w0.z, b2, acc[0]);
    acc[1] = MFMA32(w1.z, b2, acc[1]);
    acc[0] = MFMA32(w0.w, b3, acc[0]);
    acc[1] = MFMA32(w1.w, b3, acc[1]);
  }
}

// acc[mo] += sum_s frag(seg, mo, s) * src[s>>4][s&15]   (K = 64 chained units)
template <int MO>
__device__ inline void chain(const float* lds, int seg, const f32x16* src, int lane, f32x16* acc) {
#pragma unroll
  for (int s4 = 0; s4 < 8; ++s4) {
#pragma unroll
    for (int mo = 0; mo < MO; ++mo) {
      const float4 w = frag4(lds, seg, 32, mo, s4, lane);
      const int s = 4 * s4;
      acc[mo] = MFMA32(w.x, src[(s + 0) >> 4][(s + 0) & 15], acc[mo]);
      acc[mo] = MFMA32(w.y, src[(s + 1) >> 4][(s + 1) & 15], acc[mo]);
      acc[mo] = MFMA32(w.z, src[(s + 2) >> 4][(s + 2) & 15], acc[mo]);
      acc[mo] = MFMA32(w.w, src[(s + 3) >> 4][(s + 3) & 15], acc[mo]);
    }
  }
}

// tanh in ~10 VALU ops (ocml tanhf is ~3x longer and sits on the MFMA chain's
// critical path): odd Taylor polynomial for |x| < 0.125 (rel. err < 1e-9), else
// 1 - 2/(exp(2|x|)+1) with v_exp_f32 / v_rcp_f32 (abs. err ~1e-7); saturates to
// +-1, propagates NaN.
// Every multiply-add is an explicit fmaf, so the rounding never depends on the
// compiler's contraction choice: each kernel instantiation that evaluates the same
// activation gets the same bits (the activation cache is bitwise transparent).
__device__ inline float tanh_fast(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  float q = fmaf(x2, -0.0539682545f, 0.133333340f);
  q = fmaf(x2, q, -0.333333343f);
  q = fmaf(x2, q, 1.f);
  const float p = x * q;
  const float e = __expf(2.f * ax);
  const float t = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  const float r = copysignf(t, x);
  return ax < 0.125f ? p : r;
}

// tanh_fast of two values with packed f32 math (v_pk_mul / v_pk_fma / v_pk_add for the
// polynomial, the exponent argument and the reciprocal's affine step): the same IEEE
// operations in the same order as tanh_fast, so every element has tanh_fast's bits
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 tanh_fast2(f32x2 x) {
  const f32x2 ax = __builtin_elementwise_abs(x);
  const f32x2 x2 = x * x;
  f32x2 q = __builtin_elementwise_fma(x2, (f32x2)(-0.0539682545f), (f32x2)(0.133333340f));
  q = __builtin_elementwise_fma(x2, q, (f32x2)(-0.333333343f));
  q = __builtin_elementwise_fma(x2, q, (f32x2)(1.f));
  const f32x2 p = x * q;
  const f32x2 y = (ax + ax) * (f32x2)(__uint_as_float(0x3fb8aa3bu));  // __expf(2|x|) = exp2(2|x| log2 e)
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(y.x);
  e.y = __builtin_amdgcn_exp2f(y.y);
  const f32x2 d = e + (f32x2)(1.f);
  f32x2 r;
  r.x = __builtin_amdgcn_rcpf(d.x);
  r.y = __builtin_amdgcn_rcpf(d.y);
  const f32x2 t = __builtin_elementwise_fma((f32x2)(-2.f), r, (f32x2)(1.f));
  f32x2 o;
  o.x = ax.x < 0.125f ? p.x : copysignf(t.x, x.x);
  o.y = ax.y < 0.125f ? p.y : copysignf(t.y, x.y);
  return o;
}

// The exact three-way bf16 split of two f32 values (v = a + c + e exactly: RNE parts,
// each remainder exact by Sterbenz, the last one has <= 8 significant bits): one
// v_cvt_pk_bf16_f32 per part pair, the widening and the remainders on packed f32.  The
// split-operand products (mlp_split.hip, the hybrid VJP) take f32 operands as these parts.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ inline void split2(f32x2 v, bf16x2& a, bf16x2& c, bf16x2& e) {
  a = __builtin_convertvector(v, bf16x2);
  const f32x2 r = v - __builtin_convertvector(a, f32x2);
  c = __builtin_convertvector(r, bf16x2);
  e = __builtin_convertvector(r - __builtin_convertvector(c, f32x2), bf16x2);
}
// the three parts of four values (one 16x16 f32 MFMA accumulator tile of a lane)
__device__ inline void split4(const f32x4& v, bf16x4* p) {
  bf16x2 a0, c0, e0, a1, c1, e1;
  split2(f32x2{v[0], v[1]}, a0, c0, e0);
  split2(f32x2{v[2], v[3]}, a1, c1, e1);
  p[0] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3);
  p[1] = __builtin_shufflevector(c0, c1, 0, 1, 2, 3);
  p[2] = __builtin_shufflevector(e0, e1, 0, 1, 2, 3);
}
__device__ inline bf16x8 cat4(const bf16x4& lo, const bf16x4& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// The three parts of four values laid out [p0 | p1 | p2 | p0] (8 registers): its 8-element
// windows at 0 (p0, p1) and 8 (p2, p0) are K-stacked operands of a 16x16x32 product whose
// K is 4 rows x 2 parts, so the six part products i + j <= 2 of two such operands h, g take
// three MFMAs on register windows, no operand copies:
//   W8(h) W0(g) = h2 g0 + h0 g1,   W0(h) W8(g) = h0 g2 + h1 g0,   W0(h) W0(g) = h0 g0 + h1 g1
typedef __bf16 bf16x16 __attribute__((ext_vector_type(16)));
__device__ inline bf16x16 split4w(const f32x4& v) {
  bf16x2 a0, c0, e0, a1, c1, e1;
  split2(f32x2{v[0], v[1]}, a0, c0, e0);
  split2(f32x2{v[2], v[3]}, a1, c1, e1);
  const bf16x4 p0 = __builtin_shufflevector(a0, a1, 0, 1, 2, 3);
  const bf16x4 p1 = __builtin_shufflevector(c0, c1, 0, 1, 2, 3);
  const bf16x4 p2 = __builtin_shufflevector(e0, e1, 0, 1, 2, 3);
  return __builtin_shufflevector(cat4(p0, p1), cat4(p2, p0), 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14,
                                 15);
}
__device__ inline bf16x8 W0(const bf16x16& w) { return __builtin_shufflevector(w, w, 0, 1, 2, 3, 4, 5, 6, 7); }
__device__ inline bf16x8 W8(const bf16x16& w) { return __builtin_shufflevector(w, w, 8, 9, 10, 11, 12, 13, 14, 15); }

// tanh' from the activation, 1 - h^2, as one explicit fma (see tanh_fast)
__device__ inline float dtanh(float h) { return fmaf(-h, h, 1.f); }
#ifndef MRL_PK_DTANH  // 1: tile products with tanh' on packed f32 pairs
#define MRL_PK_DTANH 1
#endif
// t[r] *= 1 - h[r]^2 over a 16-float C tile: v_pk_fma / v_pk_mul on pairs, each
// element rounded exactly as t[r] * dtanh(h[r])
__device__ inline void mul_dtanh16(f32x16& t, const f32x16& h) {
#if MRL_PK_DTANH
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const f32x2 hh = f32x2{h[r], h[r + 1]};
    const f32x2 d = __builtin_elementwise_fma(-hh, hh, (f32x2)(1.f));
    const f32x2 tt = f32x2{t[r], t[r + 1]} * d;
    t[r] = tt.x;
    t[r + 1] = tt.y;
  }
#else
#pragma unroll
  for (int r = 0; r < 16; ++r) t[r] *= dtanh(h[r]);
#endif
}

__device__ inline void tanh16(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const f32x2 t = tanh_fast2(f32x2{a[r], a[r + 1]});
    a[r] = t.x;
    a[r + 1] = t.y;
  }
}

// Head (A <= 8 outputs) on VALU: a 32-wide MFMA tile would be >= 75 % padding.
// Lane half h holds 32 of the 64 units of its row; z[o] += sum_i hv[h][o][i]*src_i
// (broadcast ds_read_b128 within the half); head_finish adds the other half and the
// bias, so every lane of the row ends with all outputs.
__device__ inline void head_partial(const float* lds, const MlpDims& d, const f32x16* src, int h, float* z) {
  const float* w = lds + d.hv + h * (MAX_OUT * 32);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    if (o < d.A) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 wv = ld4(w + o * 32 + 4 * q);
        const int mt = q >> 2, r0 = 4 * (q & 3);
        acc = fmaf(wv.x, src[mt][r0], acc);
        acc = fmaf(wv.y, src[mt][r0 + 1], acc);
        acc = fmaf(wv.z, src[mt][r0 + 2], acc);
        acc = fmaf(wv.w, src[mt][r0 + 3], acc);
      }
      z[o] += acc;
    }
  }
}

// ---- cross-lane sums on VALU permutes only (v_permlane32/16_swap, DPP), never
// ds_bpermute.  Round 5: a ds_bpermute whose data register a packed-f32 VALU op
// (v_pk_add_f32 of SLP-vectorised head sums) had just written delivered stale values of
// the wave's last 16 lanes, run to run (tools/det_locate.py); hipcc pads
// packed-f32 -> VALU dependencies but not -> LDS ones.  The VALU permutes' hazards are
// the compiler's to pad.  Each helper is bit-identical to the __shfl_xor form it
// replaces (IEEE addition commutes).
// x + x(lane ^ 32)
__device__ inline float xor32_add(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
// x + x(lane ^ 16)
__device__ inline float xor16_add(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
template <int CTRL>
__device__ inline float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
// the xor butterfly over each 32-lane half, offsets 16, 8, 4, 2, 1 in that order: every
// lane of the half ends with the half's sum.  Offset 8 is row_ror:8 (= lane ^ 8 in a
// 16-lane row); offset 4 is row_ror:4, which reads lane ^ 4 or (lane ^ 4) ^ 8 -- equal
// values once the ^8 stage has run; offsets 2 and 1 are quad_perm
__device__ inline float half_sum(float x) {
  x = xor16_add(x);
  x += dpp_f<0x128>(x);  // row_ror:8
  x += dpp_f<0x124>(x);  // row_ror:4
  x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
  return x;
}

__device__ inline void head_finish(const float* lds, const MlpDims& d, float* z) {
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o)
    if (o < d.A) z[o] = xor32_add(z[o]) + lds[d.hb + o];
}

// head partial from ONE 32-unit M-tile (mt) of a layer-2 activation
__device__ inline void head_partial_mt(const float* lds, const MlpDims& d, const f32x16& src, int mt, int h,
                                       float* z) {
  const float* w = lds + d.hv + h * (MAX_OUT * 32) + mt * 16;
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    if (o < d.A) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 wv = ld4(w + o * 32 + 4 * q);
        acc = fmaf(wv.x, src[4 * q], acc);
        acc = fmaf(wv.y, src[4 * q + 1], acc);
        acc = fmaf(wv.z, src[4 * q + 2], acc);
        acc = fmaf(wv.w, src[4 * q + 3], acc);
      }
      z[o] += acc;
    }
  }
}

// acc += sum_s frag(seg, mo, s) * src[s>>4][s&15] for ONE output M-tile
__device__ inline void chain1(const float* lds, int seg, int mo, const f32x16* src, int lane, f32x16& acc) {
#pragma unroll
  for (int s4 = 0; s4 < 8; ++s4) {
    const float4 w = frag4(lds, seg, 32, mo, s4, lane);
    const int s = 4 * s4;
    acc = MFMA32(w.x, src[(s + 0) >> 4][(s + 0) & 15], acc);
    acc = MFMA32(w.y, src[(s + 1) >> 4][(s + 1) & 15], acc);
    acc = MFMA32(w.z, src[(s + 2) >> 4][(s + 2) & 15], acc);
    acc = MFMA32(w.w, src[(s + 3) >> 4][(s + 3) & 15], acc);
  }
}

// ---- primal activation cache: the forward of one theta is shared by the 11 Fisher
// products of an update (and by the VJP that follows a loss pass).  Per 32-row tile
// and lane: h1[2][16], h2[2][16] in register order, as 16 float4 groups interleaved
// over the 64 lanes (group q of tile t at ((t*16 + q)*64 + lane)*4): every wave load
// or store instruction moves 1 KB contiguous.
constexpr int CACHE_TILE_FLOATS = 64 * 64;
__device__ inline void cache_store(float* tile, int lane, int slot, const f32x16& v) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    reinterpret_cast<float4*>(tile)[(slot * 4 + q) * 64 + lane] =
        make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}
__device__ inline void cache_load(const float* tile, int lane, int slot, f32x16& v) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 x = reinterpret_cast<const float4*>(tile)[(slot * 4 + q) * 64 + lane];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
}

// forward to the head outputs only, layer 2 one M-tile at a time (h2 never fully live);
// cache != nullptr: also store h1 / h2 of the tile (slots 0,1 / 2,3)
template <class XL>
__device__ inline void forward_head_lowreg(const float* lds, const MlpDims& d, const XL& xl, int lane, float* z,
                                           float* cache = nullptr) {
  const int h = lane >> 5;
  f32x16 h1[2];
  h1[0] = load_bias16(lds, d.fb0, 0, h);
  h1[1] = load_bias16(lds, d.fb0, 1, h);
  layer0(lds, d, xl, lane, h1);
  tanh16(h1[0]);
  tanh16(h1[1]);
  if (cache != nullptr) {
    cache_store(cache, lane, 0, h1[0]);
    cache_store(cache, lane, 1, h1[1]);
  }
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) z[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    f32x16 a = load_bias16(lds, d.fb1, mo, h);
    chain1(lds, d.fa1, mo, h1, lane, a);
    __builtin_amdgcn_sched_barrier(0);
    tanh16(a);
    if (cache != nullptr) cache_store(cache, lane, 2 + mo, a);
    head_partial_mt(lds, d, a, mo, h, z);
    __builtin_amdgcn_sched_barrier(0);
  }
  head_finish(lds, d, z);
}

// JVP to the head from the cached primal activations: no primal chain is recomputed
// (the head outputs z come from the cached h2 on the VALU)
template <class XL>
// need_z = false (DiagGauss Fisher metric: 1/sigma^2, independent of the mean) skips
// the primal head, z is left 0
__device__ inline void jvp_head_cached(const float* lds, const float* ldt, const MlpDims& d, const XL& xl, int lane,
                                       const float* cache, float* z, float* dz, bool need_z = true) {
  const int h = lane >> 5;
  f32x16 h1[2], dh1[2];
  cache_load(cache, lane, 0, h1[0]);
  cache_load(cache, lane, 1, h1[1]);
  dh1[0] = load_bias16(ldt, d.fb0, 0, h);
  dh1[1] = load_bias16(ldt, d.fb0, 1, h);
  layer0(ldt, d, xl, lane, dh1);
#pragma unroll
  for (int m = 0; m < 2; ++m) mul_dtanh16(dh1[m], h1[m]);
  float dzt[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    z[o] = 0.f;
    dz[o] = 0.f;
    dzt[o] = 0.f;
  }
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    f32x16 a;
    cache_load(cache, lane, 2 + mo, a);
    f32x16 da = load_bias16(ldt, d.fb1, mo, h);
    chain1(lds, d.fa1, mo, dh1, lane, da);
    __builtin_amdgcn_sched_barrier(0);
    chain1(ldt, d.fa1, mo, h1, lane, da);
    __builtin_amdgcn_sched_barrier(0);
    mul_dtanh16(da, a);
    if (need_z) head_partial_mt(lds, d, a, mo, h, z);
    head_partial_mt(lds, d, da, mo, h, dz);
    head_partial_mt(ldt, d, a, mo, h, dzt);
  }
  if (need_z) head_finish(lds, d, z);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) dz[o] += dzt[o];
  head_finish(ldt, d, dz);
}

// forward + JVP to the head, layer 2 one M-tile at a time (peak: h1, dh1 + 2 tiles)
template <class XL>
__device__ inline void forward_jvp_head_lowreg(const float* lds, const float* ldt, const MlpDims& d, const XL& xl,
                                               int lane, float* z, float* dz) {
  const int h = lane >> 5;
  f32x16 h1[2], dh1[2];
  h1[0] = load_bias16(lds, d.fb0, 0, h);
  h1[1] = load_bias16(lds, d.fb0, 1, h);
  layer0(lds, d, xl, lane, h1);
  dh1[0] = load_bias16(ldt, d.fb0, 0, h);
  dh1[1] = load_bias16(ldt, d.fb0, 1, h);
  layer0(ldt, d, xl, lane, dh1);
  tanh16(h1[0]);
  tanh16(h1[1]);
#pragma unroll
  for (int m = 0; m < 2; ++m) mul_dtanh16(dh1[m], h1[m]);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    z[o] = 0.f;
    dz[o] = 0.f;
  }
  float dzt[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) dzt[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    f32x16 a = load_bias16(lds, d.fb1, mo, h);
    f32x16 da = load_bias16(ldt, d.fb1, mo, h);
    // scheduling fences keep each chain's fragment prefetch within 32 registers
    chain1(lds, d.fa1, mo, h1, lane, a);
    __builtin_amdgcn_sched_barrier(0);
    chain1(lds, d.fa1, mo, dh1, lane, da);
    __builtin_amdgcn_sched_barrier(0);
    chain1(ldt, d.fa1, mo, h1, lane, da);
    __builtin_amdgcn_sched_barrier(0);
    tanh16(a);
    mul_dtanh16(da, a);
    head_partial_mt(lds, d, a, mo, h, z);
    head_partial_mt(lds, d, da, mo, h, dz);
    head_partial_mt(ldt, d, a, mo, h, dzt);
  }
  head_finish(lds, d, z);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) dz[o] += dzt[o];
  head_finish(ldt, d, dz);
}

struct Fwd {
  f32x16 h1[2], h2[2];
  float z[MAX_OUT];
};

// input layer from preloaded operands x0[s] = x[row][2s+h] (KS0p <= 16)
__device__ inline void layer0_pre(const float* lds, const MlpDims& d, const float* x0, int lane, f32x16* acc) {
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    if (s4 < d.KS0p / 4) {
      const float4 w0 = frag4(lds, d.fa0, d.KS0p, 0, s4, lane);
      const float4 w1 = frag4(lds, d.fa0, d.KS0p, 1, s4, lane);
      acc[0] = MFMA32(w0.x, x0[4 * s4 + 0], acc[0]);
      acc[1] = MFMA32(w1.x, x0[4 * s4 + 0], acc[1]);
      acc[0] = MFMA32(w0.y, x0[4 * s4 + 1], acc[0]);
      acc[1] = MFMA32(w1.y, x0[4 * s4 + 1], acc[1]);
      acc[0] = MFMA32(w0.z, x0[4 * s4 + 2], acc[0]);
      acc[1] = MFMA32(w1.z, x0[4 * s4 + 2], acc[1]);
      acc[0] = MFMA32(w0.w, x0[4 * s4 + 3], acc[0]);
      acc[1] = MFMA32(w1.w, x0[4 * s4 + 3], acc[1]);
    }
  }
}

// forward to h1, h2 (no head) from preloaded input operands
__device__ inline void forward_tile_pre(const float* lds, const MlpDims& d, const float* x0, int lane, Fwd& f) {
  const int h = lane >> 5;
  f.h1[0] = load_bias16(lds, d.fb0, 0, h);
  f.h1[1] = load_bias16(lds, d.fb0, 1, h);
  layer0_pre(lds, d, x0, lane, f.h1);
  tanh16(f.h1[0]);
  tanh16(f.h1[1]);
  f.h2[0] = load_bias16(lds, d.fb1, 0, h);
  f.h2[1] = load_bias16(lds, d.fb1, 1, h);
  chain<2>(lds, d.fa1, f.h1, lane, f.h2);
  tanh16(f.h2[0]);
  tanh16(f.h2[1]);
}

template <bool HEAD, class XL>
__device__ inline void forward_tile(const float* lds, const MlpDims& d, const XL& xl, int lane, Fwd& f) {
  const int h = lane >> 5;
  f.h1[0] = load_bias16(lds, d.fb0, 0, h);
  f.h1[1] = load_bias16(lds, d.fb0, 1, h);
  layer0(lds, d, xl, lane, f.h1);
  tanh16(f.h1[0]);
  tanh16(f.h1[1]);
  f.h2[0] = load_bias16(lds, d.fb1, 0, h);
  f.h2[1] = load_bias16(lds, d.fb1, 1, h);
  chain<2>(lds, d.fa1, f.h1, lane, f.h2);
  tanh16(f.h2[0]);
  tanh16(f.h2[1]);
  if (HEAD) {
#pragma unroll
    for (int o = 0; o < MAX_OUT; ++o) f.z[o] = 0.f;
    head_partial(lds, d, f.h2, h, f.z);
    head_finish(lds, d, f.z);
  }
}

// forward + JVP along the tangent image `ldt` (same layout), interleaved layer by
// layer so h1/dh1 die before layer 2's accumulators are live.  Leaves h2 in f.h2,
// the outputs in f.z and their directional derivative in dz.
template <class XL>
__device__ inline void forward_jvp_tile(const float* lds, const float* ldt, const MlpDims& d, const XL& xl, int lane,
                                        Fwd& f, float* dz) {
  const int h = lane >> 5;
  f32x16 dh[2];
  f.h1[0] = load_bias16(lds, d.fb0, 0, h);
  f.h1[1] = load_bias16(lds, d.fb0, 1, h);
  layer0(lds, d, xl, lane, f.h1);
  dh[0] = load_bias16(ldt, d.fb0, 0, h);
  dh[1] = load_bias16(ldt, d.fb0, 1, h);
  layer0(ldt, d, xl, lane, dh);
  tanh16(f.h1[0]);
  tanh16(f.h1[1]);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[m][r] *= dtanh(f.h1[m][r]);
  f32x16 da[2];
  f.h2[0] = load_bias16(lds, d.fb1, 0, h);
  f.h2[1] = load_bias16(lds, d.fb1, 1, h);
  chain<2>(lds, d.fa1, f.h1, lane, f.h2);
  da[0] = load_bias16(ldt, d.fb1, 0, h);
  da[1] = load_bias16(ldt, d.fb1, 1, h);
  chain<2>(lds, d.fa1, dh, lane, da);
  chain<2>(ldt, d.fa1, f.h1, lane, da);
  tanh16(f.h2[0]);
  tanh16(f.h2[1]);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) da[m][r] *= dtanh(f.h2[m][r]);
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) {
    f.z[o] = 0.f;
    dz[o] = 0.f;
  }
  head_partial(lds, d, f.h2, h, f.z);
  head_finish(lds, d, f.z);
  head_partial(lds, d, da, h, dz);
  head_partial(ldt, d, f.h2, h, dz);
  head_finish(ldt, d, dz);
}

// 16-lane-row exchange (v_permlane32_swap + v_permlane16_swap, no LDS): out[q] = v of
// the lane in row q (lanes 16q .. 16q+15) with this lane's column (lane & 15).  All
// lanes active.
__device__ inline void quads_u32(uint32_t x, uint32_t* out) {
  const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // [x0 x1 x0 x1], [x2 x3 x2 x3]
  const auto a = __builtin_amdgcn_permlane16_swap(p[0], p[0], false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(p[1], p[1], false, false);
  out[0] = a[0];
  out[1] = a[1];
  out[2] = b[0];
  out[3] = b[1];
}
__device__ inline void quads(double v, double* out) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  uint32_t lo[4], hi[4];
  quads_u32((uint32_t)b, lo);
  quads_u32((uint32_t)(b >> 32), hi);
#pragma unroll
  for (int q = 0; q < 4; ++q) out[q] = __longlong_as_double((long long)(((uint64_t)hi[q] << 32) | (uint64_t)lo[q]));
}
// (v_row0 + v_row1) + (v_row2 + v_row3) for this lane's column, identical in all rows
__device__ inline float quad_sum(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float t = __uint_as_float(p[0]) + __uint_as_float(p[1]);  // rows 0,1: v0+v1; rows 2,3: v2+v3
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// the same for a double: both 32-bit halves follow the float pattern
__device__ inline double quad_sum_d(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const auto plo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
  const auto phi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
  const double t = __longlong_as_double((long long)(((uint64_t)phi[0] << 32) | plo[0])) +
                   __longlong_as_double((long long)(((uint64_t)phi[1] << 32) | plo[1]));
  const uint64_t tb = (uint64_t)__double_as_longlong(t);
  const auto qlo = __builtin_amdgcn_permlane32_swap((uint32_t)tb, (uint32_t)tb, false, false);
  const auto qhi = __builtin_amdgcn_permlane32_swap((uint32_t)(tb >> 32), (uint32_t)(tb >> 32), false, false);
  return __longlong_as_double((long long)(((uint64_t)qhi[0] << 32) | qlo[0])) +
         __longlong_as_double((long long)(((uint64_t)qhi[1] << 32) | qlo[1]));
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// the xor butterfly over the wave, offsets 32 .. 1 (every lane ends with the sum)
__device__ inline float wave_sumf(float v) { return half_sum(xor32_add(v)); }

}  // namespace mrl
