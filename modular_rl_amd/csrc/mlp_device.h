// Device building blocks shared by the MLP kernels and the rollout kernel:
// LDS fragment reads, the MFMA layer chains of the transposed-activation layout
// (see mlp_layout.h) and small wave utilities.
#pragma once
#include "mlp_layout.h"

namespace mrl {

// ------------------------------------------------------------------ device helpers
__device__ inline f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ inline float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

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
  __device__ inline float operator()(int k) const {
    if (!valid) return 0.f;
    if (k < n_obs) return x[row * n_obs + k];
    if (ept != nullptr && k == n_obs) return (float)((double)ept[row] / ts_limit);
    return 0.f;
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
__device__ inline float tanh_fast(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  const float p = x * (1.f + x2 * (-0.333333343f + x2 * (0.133333340f + x2 * -0.0539682545f)));
  const float e = __expf(2.f * ax);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  const float r = copysignf(t, x);
  return ax < 0.125f ? p : r;
}

__device__ inline void tanh16(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = tanh_fast(a[r]);
}

struct Fwd {
  f32x16 h1[2], h2[2], z;
};

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
    f.z = load_bias16(lds, d.fb2, 0, h);
    chain<1>(lds, d.fa2, f.h2, lane, &f.z);
  }
}

// JVP along the tangent image `ldt` (same layout), primal activations in f
template <class XL>
__device__ inline f32x16 jvp_tile(const float* lds, const float* ldt, const MlpDims& d, const XL& xl, int lane,
                                  const Fwd& f) {
  const int h = lane >> 5;
  f32x16 dh1[2], dh2[2];
  dh1[0] = load_bias16(ldt, d.fb0, 0, h);
  dh1[1] = load_bias16(ldt, d.fb0, 1, h);
  layer0(ldt, d, xl, lane, dh1);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) dh1[m][r] *= (1.f - f.h1[m][r] * f.h1[m][r]);
  dh2[0] = load_bias16(ldt, d.fb1, 0, h);
  dh2[1] = load_bias16(ldt, d.fb1, 1, h);
  chain<2>(lds, d.fa1, dh1, lane, dh2);
  chain<2>(ldt, d.fa1, f.h1, lane, dh2);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) dh2[m][r] *= (1.f - f.h2[m][r] * f.h2[m][r]);
  f32x16 dz = load_bias16(ldt, d.fb2, 0, h);
  chain<1>(lds, d.fa2, dh2, lane, &dz);
  chain<1>(ldt, d.fa2, f.h2, lane, &dz);
  return dz;
}

// head outputs o < 8 live in register o&3 of lane half o>>2: give every lane all 8
__device__ inline void head_gather(const f32x16& z, int lane, float* out) {
  const int h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float mine = z[r];
    const float other = __shfl_xor(mine, 32);
    out[r] = h ? other : mine;
    out[4 + r] = h ? mine : other;
  }
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline float wave_sumf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace mrl
