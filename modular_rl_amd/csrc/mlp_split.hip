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
// the six products a_i.b_j with i + j <= 2 (each exact in f32); the three dropped ones,
// a1.b2, a2.b1, a2.b2, are each <= 2^-25 |a.b|, below one f32 ulp.
// The parts are accumulated smallest first, 16 k-terms per MFMA (fewer roundings than a
// per-product f32 fma chain).  So this is fp32 arithmetic in its accuracy -- checked
// against the float64 oracle at the same 1e-4 and against the exact-f32 kernels to f32
// rounding (tests/test_gpu_split.py) -- on the bf16 matrix cores.
//
// This file holds the Fisher product's JVP half (the tangent-forward rows and the KL
// metric); its VJP half is mlp_vjp16_kernel's hybrid form (mlp_kernels.hip).  Layouts are
// those of the bf16 mode (bf16_frag.h, mlp_bf16.hip header): F tiles D[unit][row] chain
// as B fragments; the split image is the bf16 image's f32 section (biases, VALU head)
// followed by three copies of its forward bf16 section, part p at +p * PS.
// The primal activations come from the f32 activation cache of the update's SURRGRAD
// pass (mlp_kernels.hip cache layout = the F-tile register order), split on load.
#include <math.h>
#include <stdlib.h>

#include "../../include/mrl_hip.h"
#include "bf16_frag.h"
#include "mlp_device.h"
#include "rows_epilogue.h"
#include "fvp_split_role.h"

namespace mrl {

__global__ void mlp_pack_split_kernel(MlpDims d, BDims b, const float* __restrict__ th, float* __restrict__ image,
                                      int items, const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < items) split_image_item(d, b, th, image, u);
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
    void mlp_fvp_split_kernel(RowsArgs a, BDims b, const float* __restrict__ img_g, const float* __restrict__ imt_g,
                              const int32_t* __restrict__ skip) {
  split_shape<SH>(a, b);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const int W = split_fwd_words(b);  // forward segments only
  for (int i = threadIdx.x; i < W / 4; i += SPLIT_ROWS_BLOCK) {
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
    reinterpret_cast<float4*>(lds + W)[i] = reinterpret_cast<const float4*>(imt_g)[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform tile indices
  JvpSplitRole role;
  role.init(a, b, lds, lds + W, lane);
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
  const int64_t stride = (int64_t)gridDim.x * SPLIT_ROWS_WAVES;
  const int h = lane >> 5;
  int64_t tile = (int64_t)blockIdx.x * SPLIT_ROWS_WAVES + wave;
  if (tile < ntiles) role.prologue(tile);
  for (; tile < ntiles; tile += stride) {
    const int64_t tn = tile + stride < ntiles ? tile + stride : tile;  // the last tile re-reads itself
    role.tile(tile, tn, [&](bool valid, int64_t row, const float (&z)[MAX_OUT], const float (&dz)[MAX_OUT]) {
      if (valid && h == 0) row_epilogue<MRL_EPI_FVP, MAX_OUT>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
    });
  }
  (void)acc0;
  (void)acc1;
  (void)acc2;
}


// ------------------------------------------------------------------ forward rows
// The primal row passes of the fp32 update -- TRPO losses and surrogate-gradient rows
// (trpo.py:42-43, 60-64), the value prediction and the VF loss rows (core.py:611-617,
// 648-650) -- on the same split operands: layer 0 and layer 1 as six bf16 part products
// each, f32 accumulation, tanh and the A-output head on the f32 VALU.  Same per-row values
// as mlp_rows_kernel<EPI> to f32 rounding (the products are exact, the summation order
// differs); the activation cache it writes (SURRGRAD / VFLOSS, MRL_CACHE_WRITE) has the
// f32 kernel's layout, so the Fisher products and VJPs read it unchanged.
template <int SH>
__device__ inline void split_rows_shape(RowsArgs& a, BDims& b) {
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

template <int EPI, int SH>
__global__ __launch_bounds__(SPLIT_ROWS_BLOCK, 2) void mlp_rows_split_kernel(RowsArgs a, BDims b,
                                                                            const float* __restrict__ img_g,
                                                                            const int32_t* __restrict__ skip) {
  split_rows_shape<SH>(a, b);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (skip != nullptr && *skip != 0) return;
  const int W = split_fwd_words(b);
  for (int i = threadIdx.x; i < W / 4; i += SPLIT_ROWS_BLOCK)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img_g)[i];
  __syncthreads();
  const float* img = lds;
  const MlpDims dd = head_dims(a.d, b);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int A = a.A;
  float ls[MAX_OUT], sd[MAX_OUT], dls[MAX_OUT];
#pragma unroll
  for (int j = 0; j < MAX_OUT; ++j) {
    ls[j] = (a.logstd != nullptr && j < A) ? a.logstd[j] : 0.f;
    sd[j] = expf(ls[j]);
    dls[j] = 0.f;
  }
  const bool store = a.cache != nullptr && a.cache_mode == MRL_CACHE_WRITE;
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * SPLIT_ROWS_WAVES + wave; tile < ntiles;
       tile += (int64_t)gridDim.x * SPLIT_ROWS_WAVES) {
    const int64_t row = tile * 32 + (lane & 31);
    split_rows_tile<EPI>(a, b, img, dd, lane, tile, store, ls, sd, dls, acc0, acc1, acc2, a, row);
  }
  if (a.partial != nullptr) {
    acc0 = wave_sum(acc0);
    acc1 = wave_sum(acc1);
    acc2 = wave_sum(acc2);
    if (lane == 0) {
      double* p = a.partial + ((int64_t)blockIdx.x * SPLIT_ROWS_WAVES + wave) * 4;
      p[0] = acc0;
      p[1] = acc1;
      p[2] = acc2;
      p[3] = 0.0;
    }
  }
}

int launch_rows_split(int epi, int sh, const RowsArgs& a, const BDims& b, const float* image_s, int64_t blocks,
                      const int32_t* skip, void* stream) {
  const dim3 grid(blocks), blk(SPLIT_ROWS_BLOCK);
  const size_t shm = (size_t)split_fwd_words(b) * 4;
  hipStream_t s = (hipStream_t)stream;
#define MRL_RS(E, S) hipLaunchKernelGGL((mlp_rows_split_kernel<E, S>), grid, blk, shm, s, a, b, image_s, skip)
  switch (epi) {
    case MRL_EPI_PROB:
      if (sh == 1) MRL_RS(MRL_EPI_PROB, 1);
      else if (sh == 2) MRL_RS(MRL_EPI_PROB, 2);
      else if (sh == 3) MRL_RS(MRL_EPI_PROB, 3);
      else if (sh == 4) MRL_RS(MRL_EPI_PROB, 4);
      else if (sh == (3 | SH_TIME)) MRL_RS(MRL_EPI_PROB, 3 | SH_TIME);
      else if (sh == (4 | SH_TIME)) MRL_RS(MRL_EPI_PROB, 4 | SH_TIME);
      else MRL_RS(MRL_EPI_PROB, 0);
      break;
    case MRL_EPI_LOSSES:
      if (sh == 1) MRL_RS(MRL_EPI_LOSSES, 1);
      else if (sh == 2) MRL_RS(MRL_EPI_LOSSES, 2);
      else MRL_RS(MRL_EPI_LOSSES, 0);
      break;
    case MRL_EPI_SURRGRAD:
      if (sh == 1) MRL_RS(MRL_EPI_SURRGRAD, 1);
      else if (sh == 2) MRL_RS(MRL_EPI_SURRGRAD, 2);
      else MRL_RS(MRL_EPI_SURRGRAD, 0);
      break;
    case MRL_EPI_VFLOSS:
      if (sh == 3) MRL_RS(MRL_EPI_VFLOSS, 3);
      else if (sh == 4) MRL_RS(MRL_EPI_VFLOSS, 4);
      else MRL_RS(MRL_EPI_VFLOSS, 0);
      break;
    default:
      return fail(E_UNSUPPORTED, "mrl_mlp_rows_split: epilogue");
  }
#undef MRL_RS
  return hip_check(hipGetLastError(), "mrl_mlp_rows_split");
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
  return split_fwd_words(bf16_dims(d->n_in, d->n_out));
}

int mrl_mlp_pack_split(const mrl_mlp_desc* d, const float* theta, float* image, const int32_t* skip, void* stream) {
  int rc = check_desc_s(d);
  if (rc) return rc;
  if (!theta || !image) return fail(E_ARG, "null pointer");
  const MlpDims m = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  const BDims b = bf16_dims(d->n_in, d->n_out);
  const int items = b.fa0 + split_fw(b);
  hipLaunchKernelGGL(mlp_pack_split_kernel, dim3((items + 255) / 256), dim3(256), 0, (hipStream_t)stream, m, b, theta,
                     image, items, skip);
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

}  // extern "C"
