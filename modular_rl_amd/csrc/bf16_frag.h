// bf16 MFMA fragment helpers shared by the bf16 throughput mode (mlp_bf16.hip) and the
// split-operand fp32 Fisher product (mlp_split.hip): the packed bf16 image layout, the
// F-tile <-> fragment conversions and the chained layer products on
// v_mfma_f32_32x32x16_bf16.  See mlp_bf16.hip's header for the layouts.
#pragma once
#include "mlp_device.h"

namespace mrl {

// ------------------------------------------------------------------ image layout
// In 4-byte words.  f32 section: fb0, fb1 [mo][h][r], hv [h][o][mt*16 + r], hb -- the
// f32 image's biases and VALU head, same order.  bf16 section: fragments of 8 bf16
// (16 B) per lane, [frag][lane]:
//   fa0 [mo][s0]  A[i = 32mo + l%32][k = 16 s0 + 8h + j]   = W0[k][i]          (k < O)
//   fa1 [mo][s]   A[i = 32mo + l%32][k ~ u(s, h, j)]       = W1[u][i]
//   bw2 [mo]      A[i = 32mo + l%32][k = 8h + j]           = W2[i][o = k]      (o < A)
//   bt1 [no][s]   B[k ~ u(s, h, j)][col = 32no + l%32]     = W1[col][u]
// with u(s, h, j) = 32 (s >> 1) + cperm(8 (s & 1) + j, h).
struct BDims {
  int O, A, KS0B;
  int fb0, fb1, hv, hb, fa0, fa1, fwd_words, bw2, bt1, total_words;
};

__host__ __device__ constexpr BDims bf16_dims(int O, int A) {
  BDims b{};
  b.O = O;
  b.A = A;
  b.KS0B = (O + 15) / 16;
  int o = 0;
  b.fb0 = o; o += 64;
  b.fb1 = o; o += 64;
  b.hv = o; o += 2 * MAX_OUT * 32;
  b.hb = o; o += 16;
  b.fa0 = o; o += 2 * b.KS0B * 64 * 4;
  b.fa1 = o; o += 2 * 4 * 64 * 4;
  b.fwd_words = o;
  b.bw2 = o; o += 2 * 64 * 4;
  b.bt1 = o; o += 2 * 4 * 64 * 4;
  b.total_words = o;
  return b;
}

// the f32 kernels' VALU head helpers read d.hv / d.hb: point them at this image's copies
__host__ __device__ inline MlpDims head_dims(MlpDims d, const BDims& b) {
  d.hv = b.hv;
  d.hb = b.hb;
  return d;
}

__host__ __device__ inline int chain_u(int s, int h, int j) { return 32 * (s >> 1) + cperm(8 * (s & 1) + j, h); }

// bf16-section element j of fragment `frag` (lane-major within the segment)
__device__ inline float bimage_elem(const MlpDims& d, const BDims& b, const float* th, int seg, int frag, int j) {
  const int lane = frag & 63, blk = frag >> 6, i = lane & 31, h = lane >> 5;
  if (seg == 0) {  // fa0
    const int mo = blk / b.KS0B, s0 = blk % b.KS0B, k = 16 * s0 + 8 * h + j;
    return k < d.O ? th[d.tW0 + k * HID + 32 * mo + i] : 0.f;
  } else if (seg == 1) {  // fa1
    const int mo = blk >> 2, s = blk & 3;
    return th[d.tW1 + chain_u(s, h, j) * HID + 32 * mo + i];
  } else if (seg == 2) {  // bw2
    const int o = 8 * h + j;
    return o < d.A ? th[d.tW2 + (32 * blk + i) * d.A + o] : 0.f;
  } else {  // bt1
    const int no = blk >> 2, s = blk & 3;
    return th[d.tW1 + (32 * no + i) * HID + chain_u(s, h, j)];
  }
}

// ------------------------------------------------------------------ device helpers
__device__ inline bf16x8 frag_at(const float* img, int seg, int f, int lane) {
  return reinterpret_cast<const bf16x8*>(img + seg)[f * 64 + lane];
}

// registers 8s'..8s'+7 of an F (or T) tile as a bf16 fragment
__device__ inline bf16x8 pack8(const f32x16& t, int sp) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)t[8 * sp + j];
  return r;
}

// the f32 value of every register of tile mt from its two fragments (4-fragment set)
__device__ inline f32x16 unpack16(const bf16x8* fr, int mt) {
  f32x16 t;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    t[j] = (float)fr[2 * mt][j];
    t[8 + j] = (float)fr[2 * mt + 1][j];
  }
  return t;
}

// Identity B fragments.  Permuted (k ~ unit cperm(8s' + j, h) of an F tile): Xᵀ . I_perm
// turns F tile X into its T tile.  Natural (k = koff + 8h + j): turns the row operand
// A[row][k] of a k-step into the T tile D[row][k - koff ... ].
__device__ inline bf16x8 ident_perm(int sp, int lane) {
  const int c = lane & 31, h = lane >> 5;
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)(cperm(8 * sp + j, h) == c ? 1.f : 0.f);
  return r;
}
__device__ inline bf16x8 ident_nat(int koff, int lane) {
  const int c = lane & 31, h = lane >> 5;
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)(koff + 8 * h + j == c ? 1.f : 0.f);
  return r;
}

// row operand of input k-step s0: x[row][16 s0 + 8h + j] (time feature via XGlobal)
template <class XL>
__device__ inline bf16x8 x_frag(const XL& xl, int s0, int h) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)xl(16 * s0 + 8 * h + j);
  return r;
}

constexpr int MAX_KS0B = 2;  // n_in <= 32

// acc[mo] += W0-type product over the input k-steps (fa0 segment of `img`)
__device__ inline void layer0_b(const float* img, const BDims& b, const bf16x8* xb, int lane, f32x16* acc) {
#pragma unroll
  for (int s0 = 0; s0 < MAX_KS0B; ++s0) {
    if (s0 < b.KS0B) {
      acc[0] = MFMA32B(frag_at(img, b.fa0, 0 * b.KS0B + s0, lane), xb[s0], acc[0]);
      acc[1] = MFMA32B(frag_at(img, b.fa0, 1 * b.KS0B + s0, lane), xb[s0], acc[1]);
    }
  }
}

// acc += sum_s fa1[mo][s] . src[s]  (src: 4 fragments of a 64-unit F activation)
__device__ inline void chain_b(const float* img, const BDims& b, int mo, const bf16x8* src, int lane, f32x16& acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = MFMA32B(frag_at(img, b.fa1, mo * 4 + s, lane), src[s], acc);
}

}  // namespace mrl
