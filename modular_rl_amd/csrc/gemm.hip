// Tiled fp32 GEMM on v_mfma_f32_32x32x2_f32 for the wide ("layered") MLP path
// (Humanoid 376-512-512-512-17 and any hid_sizes the fused 64-wide kernels do not
// cover).  One kernel, three operand orientations, fused epilogues:
//
//   C[M,N] = sum_p op(A_p)[M,K] . op(B_p)[K,N]        p = 1 or 2 products (JVP: dX.W + X.dW)
//   op(A)(i,k) = A[i*lda + k]  (a_trans = 0)   or  A[k*lda + i]  (a_trans = 1)
//   op(B)(k,j) = B[k*ldb + j]  (b_trans = 0)   or  B[j*ldb + k]  (b_trans = 1)
//   epilogue: store | +bias | tanh(. + bias) | . * (1 - H^2) | split-K partial slab
//
// Layer forward  Y = tanh(X W + b)        NN, EPI_TANH
// JVP            dY = (1-Y^2)(dX W + X dW + db)    NN dual + bias, EPI_DTANH
// VJP input grad dX = (G W^T) (1 - X^2)    NT, EPI_DTANH
// weight grad    dW = X^T G  (K = rows)    TN, EPI_SLAB (split-K over rows, slabs reduced
//                                          by mrl_reduce_rows_f32 in fixed order)
//
// Block 128x128x32, 256 threads = 4 waves, each wave a 64x64 tile = 2x2 MFMA tiles
// (narrow 128x32 variant: 4 waves x 32x32 for head layers and small-M launches).
// Global -> registers -> LDS, double-buffered so the next tile's loads overlap the
// MFMAs.  LDS tiles are stored [row c][k] with a 36-float pitch; MFMA k-step (u, v)
// of lane half h takes tile k = 16h + 4u + v, so a lane's operands for 4 k-steps are
// one aligned ds_read_b128 and every staging write is a ds_write_b128.  Blocks are
// dealt to XCDs in contiguous tile runs; interior tiles skip all bounds checks.
#include <math.h>

#include "../../include/mrl_hip.h"
#include "mlp_device.h"
#include "rows_epilogue.h"

namespace mrl {

constexpr int GBM = 128, GBN = 128, GBK = 32, LDP = 36;  // LDP: LDS row pitch (floats)
// bf16 compute (MRL_COMPUTE_BF16): the same tiles staged as bf16 (converted, RNE, on the
// way into LDS; global operands stay fp32), pitch 40 bf16 = 80 B: the 16 rows a
// ds_read_b128 16-lane group touches land on distinct 4-bank groups.
constexpr int LDPB = 40;

struct GemmArgs {
  int64_t M, N, K;
  const float* A;
  const float* B;
  const float* A2;
  const float* B2;
  int64_t lda, ldb;
  float* C;
  int64_t ldc;
  const float* bias;
  const float* H;
  int64_t ldh;
  int epi;
  int64_t m_real;       // rows of op(A) read from memory; rows >= m_real are the ones-row
  int64_t k_chunk;      // split-K: K rows per blockIdx.z
  int64_t slab_stride;  // split-K: floats between the slabs of consecutive splits
  const int32_t* skip;
};

// One [TW x GBK] operand tile per K step (TW = 128, or 32 for the narrow tiles),
// staged global -> registers -> LDS as dst[c][k] (natural k order, pitch LDP = 36);
// c = tile row (A) or col (B).  Each thread stages TW/8 values as float4 groups of 4
// consecutive k of one c, so every LDS write is a ds_write_b128.
//  * K_CONTIG (source contiguous along k, e.g. activations [row][unit] as A): 8 lanes
//    cover one 128 B row segment -> each wave load instruction reads 8 full lines.
//  * otherwise (source contiguous along c): lanes along c, 4 coalesced scalar loads
//    (k .. k+3) per float4.
// FULL: the whole tile is in range (no per-element checks).  Rows c >= Creal of an
// in-range tile read as 1 (the ones-row of the bias gradient).
template <bool K_CONTIG, int TW>
struct Stage {
  static constexpr int NV = TW / 32;  // float4 groups per thread
  // (c, k) of float4 group w for this thread
  __device__ static inline int c_of(int t, int w) { return K_CONTIG ? (t >> 3) + 32 * w : t % TW; }
  __device__ static inline int k_of(int t, int w) { return K_CONTIG ? 4 * (t & 7) : (t / TW) * (TW / 8) + 4 * w; }
};

template <bool K_CONTIG, int TW, bool FULL>
__device__ inline void load_tile(float4 (&r)[TW / 32], const float* __restrict__ src, int64_t ld, int64_t c0,
                                 int64_t k0, int64_t C, int64_t Kend, int64_t Creal, bool vec) {
  using S = Stage<K_CONTIG, TW>;
  const int t = threadIdx.x;
#pragma unroll
  for (int w = 0; w < S::NV; ++w) {
    const int64_t gc = c0 + S::c_of(t, w), gk = k0 + S::k_of(t, w);
    float v[4];
    if (FULL) {
      if (K_CONTIG) {
        const float* p = src + gc * ld + gk;
        if (vec) {
          const float4 x = *reinterpret_cast<const float4*>(p);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = p[q];
        }
      } else {
        const float* p = src + gk * ld + gc;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = p[q * ld];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool in = gc < C && gk + q < Kend;
        const int64_t off = K_CONTIG ? gc * ld + gk + q : (gk + q) * ld + gc;
        v[q] = (in && gc < Creal) ? src[off] : (in ? 1.f : 0.f);
      }
    }
    r[w] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <bool K_CONTIG, int TW>
__device__ inline void store_tile(float* dst, const float4 (&r)[TW / 32]) {
  using S = Stage<K_CONTIG, TW>;
  const int t = threadIdx.x;
#pragma unroll
  for (int w = 0; w < S::NV; ++w)
    *reinterpret_cast<float4*>(dst + S::c_of(t, w) * LDP + S::k_of(t, w)) = r[w];
}

// split compute (MRL_COMPUTE_SPLIT): the tile's three exact bf16 parts (split2, mlp_device.h),
// part p at dst + p * part_stride, each in the bf16 tile layout
template <bool K_CONTIG, int TW>
__device__ inline void store_tile_split(__bf16* dst, int part_stride, const float4 (&r)[TW / 32]) {
  using S = Stage<K_CONTIG, TW>;
  const int t = threadIdx.x;
#pragma unroll
  for (int w = 0; w < S::NV; ++w) {
    bf16x2 a0, c0, e0, a1, c1, e1;
    split2(f32x2{r[w].x, r[w].y}, a0, c0, e0);
    split2(f32x2{r[w].z, r[w].w}, a1, c1, e1);
    __bf16* d = dst + S::c_of(t, w) * LDPB + S::k_of(t, w);
    *reinterpret_cast<bf16x4*>(d) = __builtin_shufflevector(a0, a1, 0, 1, 2, 3);
    *reinterpret_cast<bf16x4*>(d + part_stride) = __builtin_shufflevector(c0, c1, 0, 1, 2, 3);
    *reinterpret_cast<bf16x4*>(d + 2 * part_stride) = __builtin_shufflevector(e0, e1, 0, 1, 2, 3);
  }
}

template <bool K_CONTIG, int TW>
__device__ inline void store_tile_bf16(__bf16* dst, const float4 (&r)[TW / 32]) {
  using S = Stage<K_CONTIG, TW>;
  const int t = threadIdx.x;
#pragma unroll
  for (int w = 0; w < S::NV; ++w) {
    bf16x4 v;
    v[0] = (__bf16)r[w].x;
    v[1] = (__bf16)r[w].y;
    v[2] = (__bf16)r[w].z;
    v[3] = (__bf16)r[w].w;
    *reinterpret_cast<bf16x4*>(dst + S::c_of(t, w) * LDPB + S::k_of(t, w)) = v;
  }
}

// BN = 128: 2x2 waves, each a 64x64 tile (2x2 MFMA tiles).  BN = 32 (narrow heads,
// small M): 4x1 waves, each a 32x32 tile.  MODE 1 (bf16): bf16 operands
// (v_mfma_f32_32x32x16_bf16, two k-steps per 32-deep tile), f32 accumulation and
// epilogue.  MODE 2 (split, fp32-accurate): both operands split exactly into three bf16
// parts on the way into LDS, the six part products i + j <= 2 per k-step on the same bf16
// MFMA (mlp_split.hip header), f32 accumulation -- the exact-f32 kernel's results to f32
// rounding at 6 bf16 MFMAs per 16-deep k-step instead of 16 f32 ones.
template <bool AT, bool BT, int BN, int MODE>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
  constexpr bool BF = MODE != 0;
  constexpr int NP = MODE == 2 ? 3 : 1;  // bf16 parts per operand tile
  constexpr int MI = BN == 128 ? 2 : 1, NI = BN == 128 ? 2 : 1;
  // tile sizes in floats (fp32) or in 4-byte words holding two bf16 (BF; NP parts)
  constexpr int A_FL = BF ? NP * GBM * LDPB / 2 : GBM * LDP, B_FL = BF ? NP * BN * LDPB / 2 : BN * LDP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int wm = BN == 128 ? wave >> 1 : wave, wn = BN == 128 ? wave & 1 : 0;
  // XCD-aware tile order: the dispatcher deals consecutive block ids round-robin to
  // the 8 XCDs, so give each XCD a contiguous run of (m, n) tiles -- the N-tiles that
  // share one A row panel then run on the same XCD and re-read it from its L2.
  int64_t tm = blockIdx.y, tn = blockIdx.x;
  {
    const int64_t nx = gridDim.x, tiles = nx * gridDim.y;
    const int64_t L = blockIdx.x + nx * (int64_t)blockIdx.y;
    if (tiles % 8 == 0) {
      const int64_t T = (L % 8) * (tiles / 8) + L / 8;
      tm = T / nx;
      tn = T % nx;
    }
  }
  const int64_t m0 = tm * GBM, n0 = tn * BN;
  int64_t kbeg = 0, kend = g.K;
  if (g.epi == MRL_GEMM_SLAB) {
    kbeg = (int64_t)blockIdx.z * g.k_chunk;
    kend = min(g.K, kbeg + g.k_chunk);
  }
  f32x16 acc[MI][NI];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b) acc[a][b] = zero16();
  const int npairs = g.A2 != nullptr ? 2 : 1;
  const int64_t ntk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;
  const int64_t nt = npairs * ntk;
  // 16-byte loads along k need ld % 4 == 0 and 16 B aligned bases
  const bool va = !AT && (g.lda & 3) == 0 && ((reinterpret_cast<uintptr_t>(g.A) | reinterpret_cast<uintptr_t>(g.A2)) & 15) == 0;
  const bool vb = BT && (g.ldb & 3) == 0 && ((reinterpret_cast<uintptr_t>(g.B) | reinterpret_cast<uintptr_t>(g.B2)) & 15) == 0;
  // interior block: every tile in M/N range (the K tail is checked per tile)
  const bool interior = m0 + GBM <= g.m_real && n0 + BN <= g.N;
  float4 ra[GBM / 32], rb[BN / 32];
  auto load = [&](int64_t t) {
    const int p = t >= ntk ? 1 : 0;
    const int64_t k0 = kbeg + (t - p * ntk) * GBK;
    const float* Ap = p ? g.A2 : g.A;
    const float* Bp = p ? g.B2 : g.B;
    if (interior && k0 + GBK <= kend) {
      load_tile<!AT, GBM, true>(ra, Ap, g.lda, m0, k0, g.M, kend, g.m_real, va);
      load_tile<BT, BN, true>(rb, Bp, g.ldb, n0, k0, g.N, kend, g.N, vb);
    } else {
      load_tile<!AT, GBM, false>(ra, Ap, g.lda, m0, k0, g.M, kend, g.m_real, va);
      load_tile<BT, BN, false>(rb, Bp, g.ldb, n0, k0, g.N, kend, g.N, vb);
    }
  };
  if (nt > 0) load(0);
  for (int64_t t = 0; t < nt; ++t) {
    float* As = smem + (t & 1) * (A_FL + B_FL);
    float* Bs = As + A_FL;
    if constexpr (MODE == 2) {
      store_tile_split<!AT, GBM>(reinterpret_cast<__bf16*>(As), GBM * LDPB, ra);
      store_tile_split<BT, BN>(reinterpret_cast<__bf16*>(Bs), BN * LDPB, rb);
    } else if constexpr (BF) {
      store_tile_bf16<!AT, GBM>(reinterpret_cast<__bf16*>(As), ra);
      store_tile_bf16<BT, BN>(reinterpret_cast<__bf16*>(Bs), rb);
    } else {
      store_tile<!AT, GBM>(As, ra);
      store_tile<BT, BN>(Bs, rb);
    }
    __syncthreads();
    if (t + 1 < nt) load(t + 1);  // next tile's global loads overlap this tile's MFMAs
    if constexpr (MODE == 2) {
      const __bf16* Ab = reinterpret_cast<const __bf16*>(As);
      const __bf16* Bb = reinterpret_cast<const __bf16*>(Bs);
#pragma unroll
      for (int ks = 0; ks < GBK / 16; ++ks) {
        bf16x8 av[3][MI], bv[3][NI];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
            av[p][mi] = *reinterpret_cast<const bf16x8*>(Ab + p * GBM * LDPB + (wm * 32 * MI + 32 * mi + j) * LDPB +
                                                         16 * ks + 8 * h);
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            bv[p][ni] = *reinterpret_cast<const bf16x8*>(Bb + p * BN * LDPB + (wn * 32 * NI + 32 * ni + j) * LDPB +
                                                         16 * ks + 8 * h);
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {  // smallest products first
            acc[mi][ni] = MFMA32B(av[2][mi], bv[0][ni], acc[mi][ni]);
            acc[mi][ni] = MFMA32B(av[0][mi], bv[2][ni], acc[mi][ni]);
            acc[mi][ni] = MFMA32B(av[1][mi], bv[1][ni], acc[mi][ni]);
            acc[mi][ni] = MFMA32B(av[1][mi], bv[0][ni], acc[mi][ni]);
            acc[mi][ni] = MFMA32B(av[0][mi], bv[1][ni], acc[mi][ni]);
            acc[mi][ni] = MFMA32B(av[0][mi], bv[0][ni], acc[mi][ni]);
          }
      }
      continue;
    }
    if constexpr (BF) {
      // k-step s of lane half h: tile k = 16s + 8h + j (A and B agree, any order is valid)
      const __bf16* Ab = reinterpret_cast<const __bf16*>(As);
      const __bf16* Bb = reinterpret_cast<const __bf16*>(Bs);
#pragma unroll
      for (int ks = 0; ks < GBK / 16; ++ks) {
        bf16x8 av[MI], bv[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          av[mi] = *reinterpret_cast<const bf16x8*>(Ab + (wm * 32 * MI + 32 * mi + j) * LDPB + 16 * ks + 8 * h);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          bv[ni] = *reinterpret_cast<const bf16x8*>(Bb + (wn * 32 * NI + 32 * ni + j) * LDPB + 16 * ks + 8 * h);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA32B(av[mi], bv[ni], acc[mi][ni]);
      }
      continue;
    }
    // MFMA k-step (u, v) of lane half h covers tile k = 16h + 4u + v (any k->step
    // assignment is valid when A and B agree): one ds_read_b128 per operand per 4 steps
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float4 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const float4*>(As + (wm * 32 * MI + 32 * mi + j) * LDP + h * 16 + 4 * u);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const float4*>(Bs + (wn * 32 * NI + 32 * ni + j) * LDP + h * 16 + 4 * u);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          acc[mi][ni] = MFMA32(av[mi].x, bv[ni].x, acc[mi][ni]);
          acc[mi][ni] = MFMA32(av[mi].y, bv[ni].y, acc[mi][ni]);
          acc[mi][ni] = MFMA32(av[mi].z, bv[ni].z, acc[mi][ni]);
          acc[mi][ni] = MFMA32(av[mi].w, bv[ni].w, acc[mi][ni]);
        }
    }
  }
  // epilogue: lane holds column j, rows cperm(r, h) of each 32x32 tile
  float* C = g.C;
  if (g.epi == MRL_GEMM_SLAB) C += (int64_t)blockIdx.z * g.slab_stride;
  const bool full_out = m0 + GBM <= g.M && n0 + BN <= g.N;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int64_t col = n0 + wn * 32 * NI + ni * 32 + j;
      const int64_t rbase = m0 + wm * 32 * MI + mi * 32;
      if (full_out) {
        // interior tile: no per-element checks, the 16 H loads are issued together
        const float bv = g.bias != nullptr ? g.bias[col] : 0.f;
        float hv[16];
        if (g.epi == MRL_GEMM_DTANH) {
#pragma unroll
          for (int r = 0; r < 16; ++r) hv[r] = g.H[(rbase + cperm(r, h)) * g.ldh + col];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[mi][ni][r] + bv;
          if (g.epi == MRL_GEMM_TANH) v = tanh_fast(v);
          else if (g.epi == MRL_GEMM_DTANH) v *= dtanh(hv[r]);
          C[(rbase + cperm(r, h)) * g.ldc + col] = v;
        }
        continue;
      }
      if (col >= g.N) continue;
      const float bv = g.bias != nullptr ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + cperm(r, h);
        if (row >= g.M) continue;
        float v = acc[mi][ni][r] + bv;
        if (g.epi == MRL_GEMM_TANH) v = tanh_fast(v);
        else if (g.epi == MRL_GEMM_DTANH) {
          const float hv = g.H[row * g.ldh + col];
          v *= dtanh(hv);
        }
        C[row * g.ldc + col] = v;
      }
    }
}

// Bias gradients: slab[z*stride + c] = sum over row chunk z of G[r, c].  64 columns per
// block (one per lane, coalesced 256 B row segments), 4 waves interleave the rows.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ G, int64_t M, int64_t N, int64_t ldg,
                                                     int64_t chunk, float* __restrict__ slab, int64_t stride,
                                                     const int32_t* __restrict__ skip) {
  __shared__ float red[4][64];
  if (skip != nullptr && *skip != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = min(M, r0 + chunk);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    const float* p = G + col;
    int64_t r = r0 + wave;
    // CB iterations of the 16-row loop below with all their loads issued first (each
    // accumulator still adds its rows in the same order): a thin G (the Gaussian head's
    // 17 log-std columns) had one load round trip per 16 rows, 0.47 ms over 1 M rows
    constexpr int CB = 8;
    for (; r + 16 * (CB - 1) + 12 < r1; r += 16 * CB) {
      float v[CB][4];
#pragma unroll
      for (int j = 0; j < CB; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[j][q] = p[(r + 16 * j + 4 * q) * ldg];
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        s0 += v[j][0];
        s1 += v[j][1];
        s2 += v[j][2];
        s3 += v[j][3];
      }
    }
    for (; r + 12 < r1; r += 16) {
      s0 += p[r * ldg];
      s1 += p[(r + 4) * ldg];
      s2 += p[(r + 8) * ldg];
      s3 += p[(r + 12) * ldg];
    }
    for (; r < r1; r += 4) s0 += p[r * ldg];
  }
  red[wave][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wave == 0 && col < N)
    slab[(int64_t)blockIdx.y * stride + col] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// X = [obs, ep_t / limit] for the value net's time feature (core.py:659-660)
template <typename I>
__global__ void concat_time_kernel(const float* __restrict__ obs, const int32_t* __restrict__ ept, int64_t n, int O,
                                   double limit, float* __restrict__ X) {
  // I: 32-bit element indices when the output fits (the row / column split is one
  // 32-bit division instead of a 64-bit one per element)
  const I total = (I)(n * (O + 1)), w = (I)(O + 1);
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const I r = i / w, c = i - r * w;
    X[i] = c < (I)O ? obs[(int64_t)r * O + c] : (float)((double)ept[r] / limit);
  }
}

// Per-row head epilogue of the layered path: z (and dz) rows come from the last GEMM.
template <int EPI, int MA>
__global__ __launch_bounds__(256) void head_rows_kernel(RowsArgs a, const float* __restrict__ zr,
                                                        const float* __restrict__ dzr, const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int A = a.A;
  float ls[MA], sd[MA], dls[MA];
#pragma unroll
  for (int j = 0; j < MA; ++j) {
    ls[j] = (a.logstd != nullptr && j < A) ? a.logstd[j] : 0.f;
    sd[j] = expf(ls[j]);
    dls[j] = (a.dlogstd != nullptr && j < A) ? a.dlogstd[j] : 0.f;
  }
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  if constexpr (EPI == MRL_EPI_PPOSGD) {
    // one minibatch (n <= 256) in one block: block-reduced kl sets the penalty slope
    __shared__ double red[4];
    const int64_t row = threadIdx.x;
    const bool valid = row < a.n;
    float z[MA], dz[MA];
#pragma unroll
    for (int j = 0; j < MA; ++j) {
      z[j] = (valid && j < A) ? zr[row * A + j] : 0.f;
      dz[j] = 0.f;
    }
    if (valid) row_epilogue<MRL_EPI_LOSSES, MA>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
    const double klw = wave_sum(acc1);
    if (lane == 0) red[wave] = klw;
    __syncthreads();
    const double kl = ((red[0] + red[1]) + (red[2] + red[3])) * a.inv_ng;
    RowsArgs b = a;
    b.kl_coeff = a.kl_coeff + (kl > a.kl_cutoff ? (float)(2.0 * a.cutoff_coeff * (kl - a.kl_cutoff)) : 0.f);
    double d0 = 0.0, d1 = 0.0, d2 = 0.0;
    if (valid) row_epilogue<MRL_EPI_PPOGRAD, MA>(b, row, z, dz, ls, sd, dls, d0, d1, d2);
  } else {
    for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < a.n; row += (int64_t)gridDim.x * 256) {
      float z[MA], dz[MA];
#pragma unroll
      for (int j = 0; j < MA; ++j) {
        z[j] = j < A ? zr[row * A + j] : 0.f;
        dz[j] = (EPI == MRL_EPI_FVP && j < A) ? dzr[row * A + j] : 0.f;
      }
      row_epilogue<EPI, MA>(a, row, z, dz, ls, sd, dls, acc0, acc1, acc2);
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

template <int MA>
static void launch_head(int epi, dim3 grid, hipStream_t s, const RowsArgs& a, const float* z, const float* dz,
                        const int32_t* skip) {
  switch (epi) {
    case MRL_EPI_PROB: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_PROB, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
    case MRL_EPI_LOSSES: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_LOSSES, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
    case MRL_EPI_SURRGRAD: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_SURRGRAD, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
    case MRL_EPI_VFLOSS: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_VFLOSS, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
    case MRL_EPI_PPOGRAD: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_PPOGRAD, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
    case MRL_EPI_PPOSGD: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_PPOSGD, MA>), dim3(1), dim3(256), 0, s, a, z, dz, skip); break;
    default: hipLaunchKernelGGL((head_rows_kernel<MRL_EPI_FVP, MA>), grid, dim3(256), 0, s, a, z, dz, skip); break;
  }
}

}  // namespace mrl

using namespace mrl;

extern "C" {

static int64_t slab_chunk(int64_t K, int64_t splits) {
  if (splits < 1) splits = 1;
  int64_t chunk = ((K + splits - 1) / splits + GBK - 1) / GBK * GBK;
  return chunk < GBK ? GBK : chunk;
}

int64_t mrl_gemm_slab_splits(int64_t k, int32_t max_splits) {
  if (k <= 0) return 1;
  const int64_t chunk = slab_chunk(k, max_splits);
  return (k + chunk - 1) / chunk;
}

// column-tile width mrl_gemm launches for a descriptor: 32 (narrow 128x32 tiles: the heads,
// n <= 32, and small-M launches with fewer than 160 wide blocks) or 128
static int gemm_tile_n(int64_t m, int64_t n, int64_t k, int32_t epilogue, int32_t req_splits) {
  int64_t splits = 1;
  if (epilogue == MRL_GEMM_SLAB) {
    const int64_t chunk = slab_chunk(k, req_splits);
    splits = k > 0 ? (k + chunk - 1) / chunk : 1;
  }
  const int64_t wide_blocks = (n + GBN - 1) / GBN * ((m + GBM - 1) / GBM) * splits;
  return (n <= 32 || wide_blocks < 160) ? 32 : 128;
}

int32_t mrl_gemm_tile_n(const mrl_gemm_desc* d) {
  if (!d || d->m <= 0 || d->n <= 0) return 0;
  return gemm_tile_n(d->m, d->n, d->k, d->epilogue, d->splits);
}

int mrl_gemm(const mrl_gemm_desc* d, const int32_t* skip, void* stream) {
  if (!d || !d->b || !d->c || (!d->a && d->m > (d->ones_row ? 1 : 0))) return fail(E_ARG, "mrl_gemm: null pointer");
  if ((d->a2 == nullptr) != (d->b2 == nullptr)) return fail(E_ARG, "mrl_gemm: a2/b2 must be both set or both null");
  if (d->epilogue < MRL_GEMM_STORE || d->epilogue > MRL_GEMM_SLAB) return fail(E_ARG, "mrl_gemm: bad epilogue");
  if (d->epilogue == MRL_GEMM_DTANH && !d->h) return fail(E_ARG, "mrl_gemm: DTANH needs h");
  if (d->compute != MRL_COMPUTE_F32 && d->compute != MRL_COMPUTE_BF16 && d->compute != MRL_COMPUTE_SPLIT)
    return fail(E_ARG, "mrl_gemm: bad compute");
  if (d->m <= 0 || d->n <= 0) return OK;
  GemmArgs g;
  g.M = d->m;
  g.N = d->n;
  g.K = d->k;
  g.A = d->a;
  g.B = d->b;
  g.A2 = d->a2;
  g.B2 = d->b2;
  g.lda = d->lda;
  g.ldb = d->ldb;
  g.C = d->c;
  g.ldc = d->ldc;
  g.bias = d->bias;
  g.H = d->h;
  g.ldh = d->ldh;
  g.epi = d->epilogue;
  g.m_real = d->m - (d->ones_row ? 1 : 0);
  g.k_chunk = d->k;
  g.slab_stride = d->slab_stride;
  g.skip = skip;
  int64_t splits = 1;
  if (g.epi == MRL_GEMM_SLAB) {
    g.k_chunk = slab_chunk(d->k, d->splits);
    splits = d->k > 0 ? (d->k + g.k_chunk - 1) / g.k_chunk : 1;
  }
  if (splits > 65535) return fail(E_ARG, "mrl_gemm: too many splits");
  hipStream_t s = (hipStream_t)stream;
  const unsigned gm = (unsigned)((g.M + GBM - 1) / GBM);
  const int mode = d->compute == MRL_COMPUTE_BF16 ? 1 : d->compute == MRL_COMPUTE_SPLIT ? 2 : 0;
#define MRL_GEMM_KERNEL(AT, BT, BNW, SHM, grid)                                                     \
  do {                                                                                              \
    if (mode == 1) hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, BNW, 1>), grid, dim3(256), SHM, s, g);     \
    else if (mode == 2) hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, BNW, 2>), grid, dim3(256), SHM, s, g); \
    else hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, BNW, 0>), grid, dim3(256), SHM, s, g);               \
  } while (0)
#define MRL_GEMM_LAUNCH(BNW, SHM)                                                                  \
  do {                                                                                             \
    const dim3 grid((unsigned)((g.N + BNW - 1) / BNW), gm, (unsigned)splits);                      \
    if (!d->a_trans && !d->b_trans) MRL_GEMM_KERNEL(false, false, BNW, SHM, grid);                 \
    else if (!d->a_trans && d->b_trans) MRL_GEMM_KERNEL(false, true, BNW, SHM, grid);              \
    else if (d->a_trans && !d->b_trans) MRL_GEMM_KERNEL(true, false, BNW, SHM, grid);              \
    else MRL_GEMM_KERNEL(true, true, BNW, SHM, grid);                                              \
  } while (0)
  // LDS per block: two stages of the A and B tiles (fp32 pitch 36; bf16 pitch 40; split: 3 parts)
  auto shm_of = [&](int bn) -> size_t {
    return mode == 0 ? 2 * (GBM + bn) * LDP * sizeof(float)
                     : (size_t)(mode == 2 ? 3 : 1) * 2 * (GBM + bn) * LDPB * sizeof(__bf16);
  };
  if (gemm_tile_n(d->m, d->n, d->k, d->epilogue, d->splits) == 32) {
    // narrow 128x32 tiles: head layers (n_out <= 32) without 128-wide MFMA waste, and
    // small-M launches (the rollout's per-step forward over E rows) with 4x the blocks
    MRL_GEMM_LAUNCH(32, shm_of(32));
  } else {
    MRL_GEMM_LAUNCH(128, shm_of(128));
  }
#undef MRL_GEMM_KERNEL
#undef MRL_GEMM_LAUNCH
  return hip_check(hipGetLastError(), "mrl_gemm");
}

int mrl_head_rows(int32_t head, int32_t n_out, int32_t epi, const float* z, const float* dz, const float* logstd,
                  const float* dlogstd, const mrl_rows_io* io, const int32_t* skip, void* stream) {
  if (!io || !z) return fail(E_ARG, "mrl_head_rows: null pointer");
  if (head < MRL_HEAD_LINEAR || head > MRL_HEAD_GAUSS) return fail(E_ARG, "bad head kind");
  if (n_out < 1 || n_out > MRL_LAYERED_MAX_OUT) return fail(E_UNSUPPORTED, "n_out must be in [1, 32]");
  if (head == MRL_HEAD_LINEAR && n_out != 1) return fail(E_ARG, "linear head needs n_out=1");
  if (head == MRL_HEAD_GAUSS && !logstd) return fail(E_ARG, "DiagGauss needs logstd");
  if (io->feat_out) return fail(E_ARG, "mrl_head_rows: no feat_out (the layered path materialises X itself)");
  switch (epi) {
    case MRL_EPI_PROB:
      if (!io->out) return fail(E_ARG, "EPI_PROB needs out");
      break;
    case MRL_EPI_LOSSES:
    case MRL_EPI_SURRGRAD:
    case MRL_EPI_PPOGRAD:
    case MRL_EPI_PPOSGD:
      if (head == MRL_HEAD_LINEAR) return fail(E_ARG, "policy epilogue on a value net");
      if (!io->act || !io->adv || !io->oldprob || !io->partial) return fail(E_ARG, "losses need act/adv/oldprob/partial");
      if (epi != MRL_EPI_LOSSES && !io->ghead) return fail(E_ARG, "gradient epilogues need ghead");
      if (epi == MRL_EPI_PPOSGD && io->n > MRL_PPO_BLOCK_ROWS) return fail(E_ARG, "PPOSGD minibatch exceeds one block");
      break;
    case MRL_EPI_VFLOSS:
      if (head != MRL_HEAD_LINEAR || !io->target || !io->ghead || !io->partial)
        return fail(E_ARG, "VFLOSS needs a linear head, target, ghead, partial");
      break;
    case MRL_EPI_FVP:
      if (!dz || !io->ghead) return fail(E_ARG, "FVP needs dz, ghead");
      if (head == MRL_HEAD_GAUSS && !dlogstd) return fail(E_ARG, "DiagGauss FVP needs dlogstd");
      break;
    default:
      return fail(E_ARG, "unknown epilogue");
  }
  if (io->n <= 0) return OK;
  RowsArgs a{};
  a.head = head;
  a.A = n_out;
  a.gh = head == MRL_HEAD_GAUSS ? 2 * n_out : n_out;
  a.n = io->n;
  a.inv_ng = io->inv_n_global;
  a.act = io->act;
  a.adv = io->adv;
  a.oldprob = io->oldprob;
  a.target = io->target;
  a.out = io->out;
  a.ghead = io->ghead;
  a.partial = io->partial;
  a.logstd = head == MRL_HEAD_GAUSS ? logstd : nullptr;
  a.dlogstd = head == MRL_HEAD_GAUSS ? dlogstd : nullptr;
  a.kl_coeff = (float)io->kl_coeff;
  a.kl_cutoff = (float)io->kl_cutoff;
  a.cutoff_coeff = (float)io->cutoff_coeff;
  a.reverse_kl = io->reverse_kl;
  const dim3 grid((unsigned)(mrl_partial_rows(io->n) / 4));
  if (n_out <= 8) launch_head<8>(epi, grid, (hipStream_t)stream, a, z, dz, skip);
  else launch_head<MRL_LAYERED_MAX_OUT>(epi, grid, (hipStream_t)stream, a, z, dz, skip);
  return hip_check(hipGetLastError(), "mrl_head_rows");
}

int mrl_colsum(const float* g, int64_t m, int64_t n, int64_t ldg, int32_t splits, float* slab, int64_t slab_stride,
               const int32_t* skip, void* stream) {
  if (!g || !slab) return fail(E_ARG, "mrl_colsum: null pointer");
  if (n <= 0) return OK;
  const int64_t S = splits < 1 ? 1 : splits;
  if (S > 65535) return fail(E_ARG, "mrl_colsum: too many splits");
  const int64_t chunk = m > 0 ? (m + S - 1) / S : 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((n + 63) / 64), (unsigned)S), dim3(256), 0, (hipStream_t)stream,
                     g, m, n, ldg, chunk, slab, slab_stride, skip);
  return hip_check(hipGetLastError(), "mrl_colsum");
}

int mrl_concat_time(const float* obs, const int32_t* ep_t, int64_t n, int32_t n_obs, double timestep_limit, float* X,
                    int32_t max_blocks, void* stream) {
  if (!obs || !ep_t || !X) return fail(E_ARG, "null pointer");
  if (n_obs < 0 || max_blocks < 0) return fail(E_ARG, "bad n_obs / max_blocks");
  if (n <= 0) return OK;
  const int64_t total = n * (n_obs + 1);
  int64_t g = (total + 255) / 256;
  const int64_t cap = max_blocks > 0 ? max_blocks : 4096;
  if (g > cap) g = cap;
  if (total + (int64_t)g * 256 < (int64_t)INT32_MAX)
    hipLaunchKernelGGL(concat_time_kernel<uint32_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, ep_t, n, n_obs,
                       timestep_limit, X);
  else
    hipLaunchKernelGGL(concat_time_kernel<int64_t>, dim3(g), dim3(256), 0, (hipStream_t)stream, obs, ep_t, n, n_obs,
                       timestep_limit, X);
  return hip_check(hipGetLastError(), "mrl_concat_time");
}

}  // extern "C"
