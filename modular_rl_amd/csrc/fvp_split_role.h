// The Fisher product's JVP half on split bf16 operands, as a per-tile role shared by the
// standalone JVP rows kernel (mlp_split.hip: mlp_fvp_split_kernel) and the one-pass
// Fisher product (mlp_kernels.hip: mlp_fisher_hyb_kernel).  Exact three-way bf16 splits
// of every f32 MFMA operand, six part products on bf16 MFMA (mlp_split.hip header).
#pragma once
#include "../../include/mrl_hip.h"
#include "bf16_frag.h"
#include "mlp_device.h"
#include "rows_epilogue.h"

namespace mrl {

// Split image: the f32 section [0, fa0), then the three parts of the forward fragments
// (fa0, fa1: FW words each, part p of a forward segment at its bf16-image offset + p FW).
// Only the JVP half runs on split operands (the VJP half is mlp_vjp16_kernel's hybrid
// form, which splits its f32 image fragments itself), so there is no backward section.
__host__ __device__ constexpr int split_fw(const BDims& b) { return b.fwd_words - b.fa0; }
__host__ __device__ constexpr int split_fwd_words(const BDims& b) { return b.fa0 + 3 * split_fw(b); }

// part p (0, 1, 2) of an f32 value's exact three-way bf16 split
__device__ inline float bf16_part(float v, int p) {
  const __bf16 a = (__bf16)v;
  if (p == 0) return (float)a;
  const float r = v - (float)a;
  const __bf16 c = (__bf16)r;
  if (p == 1) return (float)c;
  return r - (float)c;
}

// The split image of th (mlp_pack_split_kernel; the CG update writes the next tangent's
// image with it, mrl_cg_update_pack), item u of split_image_items(b): items [0, fa0) are
// the f32 section's words (biases and the VALU head in the bf16 image's order), item
// fa0 + j is forward-fragment word j of all three parts (its two weights read and split
// once, the three part words written)
__device__ inline int split_image_items(const BDims& b) { return b.fa0 + split_fw(b); }

__device__ inline void split_image_item(const MlpDims& d, const BDims& b, const float* th, float* image, int u) {
  if (u < b.fa0) {
    int idx;
    if (u < b.fb1) idx = d.fb0 + (u - b.fb0);
    else if (u < b.hv) idx = d.fb1 + (u - b.fb1);
    else if (u < b.hb) idx = d.hv + (u - b.hv);
    else idx = d.hb + (u - b.hb);
    image[u] = image_value(d, th, idx);
    return;
  }
  const int FW = split_fw(b);
  const int wp = u;  // word of the bf16 image's forward section
  int seg, rel;
  if (wp < b.fa1) { seg = 0; rel = wp - b.fa0; }
  else { seg = 1; rel = wp - b.fa1; }
  const int frag = rel >> 2, q = rel & 3;
  const float lo = bimage_elem(d, b, th, seg, frag, 2 * q), hi = bimage_elem(d, b, th, seg, frag, 2 * q + 1);
#pragma unroll
  for (int part = 0; part < 3; ++part) {
    const __bf16 l = (__bf16)bf16_part(lo, part), h = (__bf16)bf16_part(hi, part);
    image[u + part * FW] =
        __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, l) | ((uint32_t)__builtin_bit_cast(uint16_t, h) << 16));
  }
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
__device__ inline void mfma_split(const float* img, int seg, int PS, int f, int lane, const bf16x8* x, f32x16& acc) {
  const bf16x8 w0 = frag_at(img, seg, f, lane), w1 = frag_at(img, seg + PS, f, lane);
  const bf16x8 w2 = frag_at(img, seg + 2 * PS, f, lane);
  acc = MFMA32B(w2, x[0], acc);
  acc = MFMA32B(w0, x[2], acc);
  acc = MFMA32B(w1, x[1], acc);
  acc = MFMA32B(w1, x[0], acc);
  acc = MFMA32B(w0, x[1], acc);
  acc = MFMA32B(w0, x[0], acc);
}

// scheduling fence between the JVP's phases (one phase's VALU splits are not
// interleaved into the previous phase's MFMA chain)
#define FVP_SPLIT_FENCE() __builtin_amdgcn_sched_barrier(0)

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

// The JVP of one 32-row tile per call (trpo.py:45-58): the head tangent along the tangent
// image imt from the cached f32 h1 / h2, then sink(valid, row, z, dz) per row of lane half
// 0 (the standalone kernel: row_epilogue FVP).  Software pipeline (SQ, round 4: 0.39 of the
// wave time parked on s_waitcnt): a tile's inputs x and h1 are loaded during the previous
// tile; at a tile's start its h2 loads are issued first, then the next tile's x / h1
// (vmcnt retires in order, so the wait for h2 before the head leaves the prefetch in flight).
struct JvpSplitRole {
  RowsArgs a;
  BDims b;
  const float* img;  // split image of theta (LDS)
  const float* imt;  // split image of the tangent (LDS)
  MlpDims dd;
  int lane, h, PS;
  bool need_z;       // the DiagGauss metric does not use the mean
  float xv[MAX_KS0B][8];
  f32x16 h1[2];

  __device__ __forceinline__ void init(const RowsArgs& a_, const BDims& b_, const float* img_, const float* imt_,
                                       int lane_) {
    a = a_;
    b = b_;
    img = img_;
    imt = imt_;
    dd = head_dims(a.d, b);
    lane = lane_;
    h = lane >> 5;
    PS = split_fw(b);
    need_z = a.head != MRL_HEAD_GAUSS;
  }
  __device__ __forceinline__ void load_xh1(int64_t t, float (&x)[MAX_KS0B][8], f32x16* hh) {
    const int64_t r = t * 32 + (lane & 31);
    XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, r, r < a.n};
#pragma unroll
    for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[s0][j] = s0 < b.KS0B ? xl(16 * s0 + 8 * h + j) : 0.f;
    cache_load(a.cache + t * CACHE_TILE_FLOATS, lane, 0, hh[0]);
    cache_load(a.cache + t * CACHE_TILE_FLOATS, lane, 1, hh[1]);
  }
  // the first tile's x / h1
  __device__ __forceinline__ void prologue(int64_t tile) { load_xh1(tile, xv, h1); }
  // tile `tile` (its x / h1 already loaded), prefetching tile tn's (tn == tile: re-read);
  // PF = false: no prefetch -- the tile's own x / h1 are loaded here, after its h2 (and no
  // prologue), so the tile's bytes all enter L2 within one round (the one-pass product's
  // VJP role re-reads them a round later: MRL_FISHER_JVP_PF)
  template <bool PF = true, class Sink>
  __device__ __forceinline__ void tile(int64_t tile, int64_t tn, Sink&& sink) {
    const int64_t row = tile * 32 + (lane & 31);
    const bool valid = row < a.n;
    const float* ct = a.cache + tile * CACHE_TILE_FLOATS;
    f32x16 h2[2];
    cache_load(ct, lane, 2, h2[0]);
    cache_load(ct, lane, 3, h2[1]);
    __builtin_amdgcn_sched_barrier(0);
    float xn[MAX_KS0B][8];
    f32x16 h1n[2];
    if constexpr (PF) load_xh1(tn, xn, h1n);
    else load_xh1(tile, xv, h1);
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
        mfma_split(imt, b.fa0, PS, 0 * b.KS0B + s0, lane, xs, dh[0]);
        mfma_split(imt, b.fa0, PS, 1 * b.KS0B + s0, lane, xs, dh[1]);
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
      mfma_split(img, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
      mfma_split(img, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
    }
    FVP_SPLIT_FENCE();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 ps[3];
      split8(h1[s >> 1], s & 1, ps);
      mfma_split(imt, b.fa1, PS, 0 * 4 + s, lane, ps, da2[0]);
      mfma_split(imt, b.fa1, PS, 1 * 4 + s, lane, ps, da2[1]);
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
    sink(valid, row, z, dz);
    if constexpr (PF) {
#pragma unroll
      for (int s0 = 0; s0 < MAX_KS0B; ++s0)
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[s0][j] = xn[s0][j];
      h1[0] = h1n[0];
      h1[1] = h1n[1];
    }
  }
};

// One 32-row tile of the forward row passes on split operands (mlp_rows_split_kernel's
// per-tile body; also the one-pass policy gradient's forward role, mlp_fisher_hyb_kernel
// PROD 1): h1 = tanh(x W0 + b0), h2 = tanh(h1 W1 + b1) with six bf16 part products per
// k-step, the head on the f32 VALU, the activation cache stored when `store`; then the
// row epilogue of lane half 0 with its arguments / row index `ae`, `erow` (the pass's own
// `a`, row -- or tile-local ones: the one-pass gradient points ghead at its LDS mailbox,
// LDSHEAD)
template <int EPI, bool LDSHEAD = false>
__device__ __forceinline__ void split_rows_tile(const RowsArgs& a, const BDims& b, const float* img, const MlpDims& dd,
                                                int lane, int64_t tile, bool store, const float (&ls)[MAX_OUT],
                                                const float (&sd)[MAX_OUT], const float (&dls)[MAX_OUT],
                                                double& acc0, double& acc1, double& acc2, const RowsArgs& ae,
                                                int64_t erow) {
  const int h = lane >> 5, PS = split_fw(b);
  const int64_t row = tile * 32 + (lane & 31);
  const bool valid = row < a.n;
  XGlobalNB xl{a.x, a.ept, a.ts_limit, a.n_obs, row, valid};
  float* ct = store ? a.cache + tile * CACHE_TILE_FLOATS : nullptr;
  // layer 0: h1 = tanh(x W0 + b0)
  f32x16 h1[2] = {load_bias16(img, b.fb0, 0, h), load_bias16(img, b.fb0, 1, h)};
#pragma unroll
  for (int s0 = 0; s0 < MAX_KS0B; ++s0) {
    if (s0 < b.KS0B) {
      float xv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = xl(16 * s0 + 8 * h + j);
      bf16x8 xs[3];
      split8v(xv, xs);
      mfma_split(img, b.fa0, PS, 0 * b.KS0B + s0, lane, xs, h1[0]);
      mfma_split(img, b.fa0, PS, 1 * b.KS0B + s0, lane, xs, h1[1]);
    }
  }
  tanh16(h1[0]);
  tanh16(h1[1]);
  if (store) {
    cache_store(ct, lane, 0, h1[0]);
    cache_store(ct, lane, 1, h1[1]);
  }
  // layer 1: h2 = tanh(h1 W1 + b1), each input fragment split once for both output tiles
  f32x16 a2[2] = {load_bias16(img, b.fb1, 0, h), load_bias16(img, b.fb1, 1, h)};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 ps[3];
    split8(h1[s >> 1], s & 1, ps);
    mfma_split(img, b.fa1, PS, 0 * 4 + s, lane, ps, a2[0]);
    mfma_split(img, b.fa1, PS, 1 * 4 + s, lane, ps, a2[1]);
  }
  FVP_SPLIT_FENCE();
  float z[MAX_OUT], dz[MAX_OUT];
#pragma unroll
  for (int o = 0; o < MAX_OUT; ++o) z[o] = dz[o] = 0.f;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    tanh16(a2[mo]);
    if (store) cache_store(ct, lane, 2 + mo, a2[mo]);
    head_partial_mt(img, dd, a2[mo], mo, h, z);
  }
  head_finish(img, dd, z);
  if constexpr (EPI == MRL_EPI_PROB)
    if (a.feat != nullptr && valid) write_feature_row(a, row, h, xl);
  if (valid && h == 0) row_epilogue<EPI, MAX_OUT, LDSHEAD>(ae, erow, z, dz, ls, sd, dls, acc0, acc1, acc2);
}

// launch mlp_rows_split_kernel<epi, sh> (mlp_split.hip) for mrl_mlp_rows_split
int launch_rows_split(int epi, int sh, const RowsArgs& a, const BDims& b, const float* image_s, int64_t blocks,
                      const int32_t* skip, void* stream);

}  // namespace mrl
