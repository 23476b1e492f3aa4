// Packed LDS "image" of a tanh MLP with two 64-wide hidden layers, laid out as
// per-lane MFMA A-operand fragments (v_mfma_f32_32x32x2_f32) so that a kernel
// copies it linearly into LDS and reads every weight fragment with one
// conflict-free ds_read_b128 per 4 k-steps.
//
// Reference net: Keras Dense(64,tanh) x2 + Dense(out) (`agentzoo.py:34-48,55-58`).
// Flat theta order (`core.py:518-557`): W0 (in,64) row-major, b0, W1 (64,64),
// b1, W2 (64,A), b2, [logstd (A) for DiagGauss].
//
// Activations are kept TRANSPOSED in MFMA accumulators: a 32-row tile of a
// 64-unit layer is two 32x32 C tiles D[unit][row] (row on the lane, units in the
// 16 registers: unit = 32*mt + cperm(r, lane>>5)).  Such a tile is directly the
// B operand of the next layer (k-step s takes register s&15 of tile s>>4, lane
// half h supplying unit 32*(s>>4) + cperm(s&15, h)), so layers chain with no data
// movement; the weight fragments below are permuted to match.
#pragma once
#include "../../include/mrl_hip.h"
#include "mrl_common.h"

namespace mrl {

constexpr int HID = 64;       // hidden width (fast path)
constexpr int MAX_IN = 32;    // input features (obs [+ time feature])
constexpr int MAX_OUT = 8;    // head outputs backpropagated
constexpr int IMG_PAD = 36;   // per-unit stride of LDS transpose scratch (floats)

struct MlpDims {
  int O, A;        // inputs, head outputs
  int KS0p;        // input-layer k-steps (ceil(O/2)) rounded up to a multiple of 4
  int fa0, fa1, fb0, fb1, hv, hb, ba1, ba2;  // segment offsets (floats)
  int fwd_size, total_size;
  // flat theta offsets
  int tW0, tb0, tW1, tb1, tW2, tb2, tls, P;
};

__host__ __device__ constexpr MlpDims mlp_dims(int O, int A, int gauss) {
  MlpDims d{};
  d.O = O;
  d.A = A;
  int ks0 = (O + 1) / 2;
  d.KS0p = (ks0 + 3) & ~3;
  int o = 0;
  d.fa0 = o; o += 2 * d.KS0p * 64;
  d.fa1 = o; o += 2 * 32 * 64;
  d.fb0 = o; o += 2 * 2 * 16;
  d.fb1 = o; o += 2 * 2 * 16;
  d.hv = o; o += 2 * MAX_OUT * 32;   // head weights for VALU: [h][o][mt*16 + r] = W2[32mt + cperm(r,h)][o]
  d.hb = o; o += 16;                 // head bias (A <= 8, padded)
  d.fwd_size = o;
  d.ba1 = o; o += 2 * 32 * 64;
  d.ba2 = o; o += 2 * 4 * 64;
  d.total_size = o;
  d.tW0 = 0;
  d.tb0 = d.tW0 + O * HID;
  d.tW1 = d.tb0 + HID;
  d.tb1 = d.tW1 + HID * HID;
  d.tW2 = d.tb1 + HID;
  d.tb2 = d.tW2 + HID * A;
  d.tls = d.tb2 + A;
  d.P = d.tls + (gauss ? A : 0);
  return d;
}

// Shapes the benchmark configs run, compiled as their own kernel instantiations so
// every dimension (inputs, outputs, head, k-steps) is a compile-time constant: no
// runtime branches on the net shape inside the tile loops.  Shape 0 = any shape,
// dimensions read at run time.  Inputs are plain rows (no time-feature column).
struct StaticShape {
  int O, A, head;
};
constexpr int N_STATIC_SHAPES = 5;
constexpr StaticShape STATIC_SHAPES[N_STATIC_SHAPES] = {
    {0, 0, 0},
    {11, 3, MRL_HEAD_GAUSS},   // Hopper-v2 policy
    {4, 2, MRL_HEAD_SOFTMAX},  // CartPole-v0 policy
    {12, 1, MRL_HEAD_LINEAR},  // Hopper-v2 value net ([obs, t / limit])
    {5, 1, MRL_HEAD_LINEAR},   // CartPole-v0 value net
};
// SH | SH_TIME: a value-net shape whose last input column is the time feature
// ep_t / limit, read beside O - 1 observation columns (the prediction pass straight
// from the rollout's rows, no materialised [obs, t] copy)
constexpr int SH_TIME = 8;
__host__ __device__ constexpr MlpDims static_dims(int sh) {
  return mlp_dims(STATIC_SHAPES[sh].O, STATIC_SHAPES[sh].A, STATIC_SHAPES[sh].head == MRL_HEAD_GAUSS);
}

// fragment slot (mo, s) of a segment with KSp k-steps -> float offset of lane 0
__host__ __device__ inline int frag_off(int mo, int s, int KSp, int lane) {
  return ((mo * (KSp / 4) + (s >> 2)) * 64 + lane) * 4 + (s & 3);
}

// k index (input unit) fed by lane half h at k-step s of a chained (64-unit) layer
__host__ __device__ inline int chain_k(int s, int h) { return 32 * (s >> 4) + cperm(s & 15, h); }

// value of image element `idx` given flat theta (nullptr => zeros)
__host__ __device__ inline float image_value(const MlpDims& d, const float* th, int idx) {
  auto dec = [&](int seg, int KSp, int& mo, int& s, int& lane) {
    int rel = idx - seg;
    int q = rel & 3;
    int l = (rel >> 2) & 63;
    int blk = rel >> 8;  // mo * (KSp/4) + s4
    mo = blk / (KSp / 4);
    s = (blk % (KSp / 4)) * 4 + q;
    lane = l;
  };
  int mo, s, lane;
  if (idx < d.fa1) {                      // FA0: A[i=out][k=in] = W0[in][out]
    dec(d.fa0, d.KS0p, mo, s, lane);
    int k = 2 * s + (lane >> 5);
    int j = 32 * mo + (lane & 31);
    return k < d.O ? th[d.tW0 + k * HID + j] : 0.f;
  } else if (idx < d.fb0) {               // FA1
    dec(d.fa1, 32, mo, s, lane);
    int k = chain_k(s, lane >> 5);
    int j = 32 * mo + (lane & 31);
    return th[d.tW1 + k * HID + j];
  } else if (idx < d.fb1) {               // FB0 [mo][h][r]
    int rel = idx - d.fb0;
    int r = rel & 15, h = (rel >> 4) & 1, m = rel >> 5;
    return th[d.tb0 + 32 * m + cperm(r, h)];
  } else if (idx < d.hv) {                // FB1
    int rel = idx - d.fb1;
    int r = rel & 15, h = (rel >> 4) & 1, m = rel >> 5;
    return th[d.tb1 + 32 * m + cperm(r, h)];
  } else if (idx < d.hb) {                // HV [h][o][mt*16 + r] = W2[32mt + cperm(r,h)][o]
    int rel = idx - d.hv;
    int i = rel & 31, o = (rel >> 5) % MAX_OUT, h = rel / (32 * MAX_OUT);
    int u = 32 * (i >> 4) + cperm(i & 15, h);
    return o < d.A ? th[d.tW2 + u * d.A + o] : 0.f;
  } else if (idx < d.fwd_size) {          // HB
    int o = idx - d.hb;
    return o < d.A ? th[d.tb2 + o] : 0.f;
  } else if (idx < d.ba2) {               // BA1: A[i=in][k=out] = W1[in][out]
    dec(d.ba1, 32, mo, s, lane);
    int i = 32 * mo + (lane & 31);
    int k = chain_k(s, lane >> 5);
    return th[d.tW1 + i * HID + k];
  } else {                                // BA2: A[i=in][k=out] = W2[in][out], out = s + 4h
    dec(d.ba2, 4, mo, s, lane);
    int i = 32 * mo + (lane & 31);
    int o = s + 4 * (lane >> 5);
    return o < d.A ? th[d.tW2 + i * d.A + o] : 0.f;
  }
}

// ------------------------------------------------------------------ rollout image
// The fused rollout step kernel is latency-bound at one wave per SIMD, so it runs 16
// envs per wave on v_mfma_f32_16x16x4_f32: a 16-row tile halves the per-wave MFMA
// chain and tanh count of the 32-row layout above.  Activations D[unit][row]: lane l
// holds row l&15 and units 16*mt + 4*(l>>4) + r (r = 0..3) of 16-unit tile mt, which
// is directly the B operand of the next layer's k-step (mt, q = r) when the k index
// of lane group g stands for unit 16*mt + 4*g + q; the weight fragments are permuted
// to match.  Every lane loads its fragments straight into registers (no LDS copy).
struct RDims {
  int KS0, KS0p;  // input-layer k-steps (4 inputs each), padded to a multiple of 4
  int a0, a1, b0, b1, hv, hb, f32_size;
  int ba0, ba1, bs1, size;  // bf16 fragments (v_mfma_f32_16x16x32_bf16): bf16 mode; bs1: split W1 (fp32)
};

__host__ __device__ constexpr RDims rollout_dims(int O) {
  RDims r{};
  r.KS0 = (O + 3) / 4;
  r.KS0p = (r.KS0 + 3) & ~3;
  int o = 0;
  r.a0 = o; o += 4 * r.KS0p * 64;   // [mo][ks>>2][lane][ks&3] = W0[4ks + (lane>>4)][16mo + (lane&15)]
  r.a1 = o; o += 4 * 16 * 64;       // [mo][mt][lane][q]       = W1[16mt + 4(lane>>4) + q][16mo + (lane&15)]
  r.b0 = o; o += 64;                // [g][4mt + r]            = b0[16mt + 4g + r]
  r.b1 = o; o += 64;                //                           b1
  r.hv = o; o += 4 * MAX_OUT * 16;  // [g][o][4mt + r]         = W2[16mt + 4g + r][o]
  r.hb = o; o += 16;                // b2 (padded)
  r.f32_size = o;
  // bf16 mode: 8 bf16 (4 words) per lane and fragment, A[i = 16mo + (l&15)][k = 8g + j]
  // (g = l >> 4): ba0 [mo][lane] = W0[k][i] (one k-step covers n_in <= 32); ba1
  // [mo][p][lane] = W1[u][i], k ~ unit u = 32p + 16(j>>2) + 4g + (j&3) -- the units lane
  // group g holds in registers r of the 16-unit activation tiles 2p, 2p+1.
  r.ba0 = o; o += 4 * 64 * 4;
  r.ba1 = o; o += 4 * 2 * 64 * 4;
  // fp32 mode: the three exact bf16 parts of the ba1 fragments, [part][mo][p][lane]: layer 1
  // of the rollout forward on split operands (six part products, f32 accumulation)
  r.bs1 = o; o += 3 * 4 * 2 * 64 * 4;
  r.size = o;
  return r;
}

__host__ __device__ inline int rb_unit(int p, int g, int j) { return 32 * p + 16 * (j >> 2) + 4 * g + (j & 3); }

// element j of bf16 fragment `frag` (ba0: frag = mo*64 + lane; ba1: (mo*2 + p)*64 + lane)
__host__ __device__ inline float rimage_bf16_elem(const MlpDims& d, const float* th, bool l1, int frag, int j) {
  const int lane = frag & 63, blk = frag >> 6, g = lane >> 4, i = lane & 15;
  if (!l1) {
    const int k = 8 * g + j;
    return k < d.O ? th[d.tW0 + k * HID + 16 * blk + i] : 0.f;
  }
  const int mo = blk >> 1, p = blk & 1;
  return th[d.tW1 + rb_unit(p, g, j) * HID + 16 * mo + i];
}

// value of rollout-image element `idx` given flat theta (layout above)
__host__ __device__ inline float rimage_value(const RDims& r, const MlpDims& d, const float* th, int idx) {
  if (idx < r.a1) {
    const int rel = idx - r.a0, q = rel & 3, lane = (rel >> 2) & 63, blk = rel >> 8;
    const int mo = blk / (r.KS0p / 4), ks = (blk % (r.KS0p / 4)) * 4 + q;
    const int k = 4 * ks + (lane >> 4), u = 16 * mo + (lane & 15);
    return k < d.O ? th[d.tW0 + k * HID + u] : 0.f;
  } else if (idx < r.b0) {
    const int rel = idx - r.a1, q = rel & 3, lane = (rel >> 2) & 63, blk = rel >> 8;
    const int mo = blk >> 2, mt = blk & 3;
    return th[d.tW1 + (16 * mt + 4 * (lane >> 4) + q) * HID + 16 * mo + (lane & 15)];
  } else if (idx < r.hv) {
    const bool first = idx < r.b1;
    const int rel = idx - (first ? r.b0 : r.b1), g = rel >> 4, i = rel & 15;
    return th[(first ? d.tb0 : d.tb1) + 16 * (i >> 2) + 4 * g + (i & 3)];
  } else if (idx < r.hb) {
    const int rel = idx - r.hv, i = rel & 15, o = (rel >> 4) % MAX_OUT, g = rel / (16 * MAX_OUT);
    return o < d.A ? th[d.tW2 + (16 * (i >> 2) + 4 * g + (i & 3)) * d.A + o] : 0.f;
  } else {
    const int o = idx - r.hb;
    return o < d.A ? th[d.tb2 + o] : 0.f;
  }
}

}  // namespace mrl
