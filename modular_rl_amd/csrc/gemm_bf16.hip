// bf16-operand GEMMs of the layered MLP path's throughput mode (MRL_COMPUTE_BF16 with
// a bf16 tape): the operands live in HBM as bf16 (half the bytes of gemm.hip's
// fp32-staged tiles), accumulation stays f32 on v_mfma_f32_32x32x16_bf16.
//
//  mrl_gemm_bf16      C[M,N] = A[M,K] . B[K,N]  (+ A2 . B2)  + bias, epilogue store |
//                     tanh | * (1 - H^2); A row-major (K contiguous), B given as its
//                     transpose Bt[N,K] (K contiguous: the packed weight images), so
//                     both tiles stage global -> LDS as whole 16-B rows segments and
//                     every MFMA operand is one ds_read_b128.  Output f32 or bf16.
//                     Layer forward (tanh), JVP (dual product, * (1 - H^2)), VJP
//                     input grad (Bt = W itself, * (1 - H^2)).
//  mrl_gemm_bf16_tn   weight gradients C[M,N] = sum_r A[r,M] B[r,N] over the rows r
//                     (K = rows, split-K into f32 slabs); A and B are row-major
//                     activations / gradients, staged row-major and read as MFMA
//                     operands with the gfx950 transposing LDS read ds_read_b64_tr_b16.
//                     The bias gradient rides as a ones-column of A.
//
// Block 128 x BN (BN = 128: 2x2 waves of 64x64; BN = 32: 4 waves of 32x32, for the
// heads), global -> registers -> LDS double-buffered (the next K step's loads are in
// flight under this step's MFMAs), blocks dealt to the XCDs in contiguous tile runs.
#include <math.h>
#include <stdlib.h>

#include "../../include/mrl_hip.h"
#include "mlp_device.h"

namespace mrl {

typedef uint16_t bfr_t;  // raw bf16 bits in memory
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

__device__ inline float bf2f(bfr_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ inline bfr_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }  // RNE

// ------------------------------------------------------------------ NN / NT (Bt) GEMM
constexpr int QBM = 128;

struct GemmB16Args {
  int64_t M, N, K;
  const bfr_t* A;
  const bfr_t* Bt;
  const bfr_t* A2;
  const bfr_t* Bt2;
  int64_t lda, ldb;
  void* C;
  int64_t ldc;
  const float* bias;
  const bfr_t* H;
  int64_t ldh;
  int epi;
  const int32_t* skip;
};

// one 16-B chunk (8 bf16 along k) of row r, k offset kc of a row-major [rows][ld]
// operand; chunks at or past K read as zero (K's padding columns are zero in memory)
__device__ inline u32x4v load_chunk(const bfr_t* __restrict__ p, int64_t r, int64_t rows, int64_t ld, int64_t kc,
                                    int64_t K) {
  if (r < rows && kc < K) return *reinterpret_cast<const u32x4v*>(p + r * ld + kc);
  return u32x4v{0u, 0u, 0u, 0u};
}

// QBK: K per LDS stage; row pitch QBK + 8 bf16 (144 B for 64, 80 B for 32): the 16
// rows a ds_read_b128 16-lane group touches start on distinct 4-bank groups
template <int BN, bool OUTBF, int QBK>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmB16Args g) {
  constexpr int QLD = QBK + 8;
  constexpr int MI = BN == 128 ? 2 : 1, NI = MI;
  constexpr int NA = QBM * (QBK / 8) / 256, NB = (BN * (QBK / 8) + 255) / 256;  // 16-B chunks per thread
  constexpr int STAGE = (QBM + BN) * QLD;                               // bf16 per LDS stage
  __shared__ __attribute__((aligned(16))) bfr_t smem[2 * STAGE];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int wm = BN == 128 ? wave >> 1 : wave, wn = BN == 128 ? wave & 1 : 0;
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
  const int64_t m0 = tm * QBM, n0 = tn * BN;
  const int64_t ntk = (g.K + QBK - 1) / QBK;
  const int64_t nt = (g.A2 != nullptr ? 2 : 1) * ntk;
  // thread t stages chunk c (k = 8c) of rows r (+ RS i)
  constexpr int CPR = QBK / 8, RS = 256 / CPR;  // chunks per row, rows per pass
  const int sc = threadIdx.x % CPR, sr = threadIdx.x / CPR;
  u32x4v ra[NA], rb[NB];
  auto load = [&](int64_t t) {
    const bool p2 = t >= ntk;
    const int64_t k0 = (t - (p2 ? ntk : 0)) * QBK + 8 * sc;
    const bfr_t* A = p2 ? g.A2 : g.A;
    const bfr_t* B = p2 ? g.Bt2 : g.Bt;
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = load_chunk(A, m0 + sr + RS * i, g.M, g.lda, k0, g.K);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = sr + RS * i < BN ? load_chunk(B, n0 + sr + RS * i, g.N, g.ldb, k0, g.K) : u32x4v{0u, 0u, 0u, 0u};
  };
  auto store = [&](bfr_t* st) {
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<u32x4v*>(st + (sr + RS * i) * QLD + 8 * sc) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (sr + RS * i < BN) *reinterpret_cast<u32x4v*>(st + (QBM + sr + RS * i) * QLD + 8 * sc) = rb[i];
  };
  f32x16 acc[MI][NI];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b) acc[a][b] = zero16();
  if (nt > 0) {
    load(0);
    store(smem);
  }
  for (int64_t t = 0; t < nt; ++t) {
    __syncthreads();
    const bfr_t* As = smem + (t & 1) * STAGE;
    const bfr_t* Bs = As + QBM * QLD;
    if (t + 1 < nt) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < QBK / 16; ++ks) {
      bf16x8 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const bf16x8*>(As + (wm * 32 * MI + 32 * mi + j) * QLD + 16 * ks + 8 * h);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 32 * NI + 32 * ni + j) * QLD + 16 * ks + 8 * h);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA32B(bv[ni], av[mi], acc[mi][ni]);  // C^T tiles
    }
    if (t + 1 < nt) store(smem + ((t + 1) & 1) * STAGE);
  }
  // epilogue: the accumulators hold C^T tiles, so lane (j, h) holds ROW j of each 32x32
  // C tile, at columns cperm(r, h): four runs of 4 consecutive columns (8q + 4h + 0..3),
  // each one 8-B (bf16) / 16-B (f32) store, bias and H loads likewise vectorised
  const bool vec = (g.ldc & 3) == 0 && (g.epi != MRL_GEMM_DTANH || (g.ldh & 3) == 0);
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int64_t row = m0 + wm * 32 * MI + mi * 32 + j;
      if (row >= g.M) continue;
      const int64_t cbase = n0 + wn * 32 * NI + ni * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t c0 = cbase + 8 * q + 4 * h;
        float v[4];
        if (vec && c0 + 4 <= g.N) {
          const float4 b = g.bias != nullptr ? *reinterpret_cast<const float4*>(g.bias + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
          v[0] = acc[mi][ni][4 * q + 0] + b.x;
          v[1] = acc[mi][ni][4 * q + 1] + b.y;
          v[2] = acc[mi][ni][4 * q + 2] + b.z;
          v[3] = acc[mi][ni][4 * q + 3] + b.w;
          if (g.epi == MRL_GEMM_TANH) {
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              const f32x2 t = tanh_fast2(f32x2{v[e], v[e + 1]});
              v[e] = t.x;
              v[e + 1] = t.y;
            }
          } else if (g.epi == MRL_GEMM_DTANH) {
            const uint2 hb = *reinterpret_cast<const uint2*>(g.H + row * g.ldh + c0);
            v[0] *= dtanh(__uint_as_float(hb.x << 16));
            v[1] *= dtanh(__uint_as_float(hb.x & 0xffff0000u));
            v[2] *= dtanh(__uint_as_float(hb.y << 16));
            v[3] *= dtanh(__uint_as_float(hb.y & 0xffff0000u));
          }
          if (OUTBF) {
            const uint2 o = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                             (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
            *reinterpret_cast<uint2*>(reinterpret_cast<bfr_t*>(g.C) + row * g.ldc + c0) = o;
          } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + row * g.ldc + c0) = make_float4(v[0], v[1], v[2], v[3]);
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t col = c0 + e;
          if (col >= g.N) continue;
          float x = acc[mi][ni][4 * q + e] + (g.bias != nullptr ? g.bias[col] : 0.f);
          if (g.epi == MRL_GEMM_TANH) x = tanh_fast(x);
          else if (g.epi == MRL_GEMM_DTANH) x *= dtanh(bf2f(g.H[row * g.ldh + col]));
          if (OUTBF) reinterpret_cast<bfr_t*>(g.C)[row * g.ldc + col] = f2bf(x);
          else reinterpret_cast<float*>(g.C)[row * g.ldc + col] = x;
        }
      }
    }
}

// ------------------------------------------------------------------ streaming NN GEMM
// For the tall layered-path GEMMs (M ~ 1 M rows, K <= 512, N = 512: HBM-bound at their
// 256 FLOP per byte) the tiled kernel above re-stages B for every 128-row tile and pays
// a prologue / epilogue per 8-step K loop.  Here B stays put and A streams:
//  * one 512-thread block per CU (persistent); its LDS holds one BN-column slice of Bt
//    for all of K (BN = 128; two 64-column slices of Bt and Bt2 for the dual product),
//    pitch KP + 8 bf16 (conflict-free ds_read_b128 fragments);
//  * each wave owns 32 rows at a time and streams their A fragments straight from
//    global memory into registers, one chunk of CK k-steps ahead of the MFMAs
//    (register double buffer; two waves per SIMD cover each other's gaps);
//  * block -> (XCD, column slice, row group): the nslice blocks that need the same A
//    rows sit on one XCD and walk the same row tiles in the same order, so each A line
//    comes from HBM once and from that XCD's L2 for the other slices (placement is a
//    speed assumption only; any placement gives the same result);
//  * epilogue as above (C^T accumulators: lane j holds row j): bias, tanh / * (1 - H^2),
//    bf16 or f32 stores.
// Same operands, same per-output k order as gemm_bf16_kernel (MFMA k-steps of 16 in
// order, one f32 accumulator per output): bit-identical results.
struct StreamPlan {
  int nslice, groups_per_xcd;
};

template <int KP, bool DUAL, bool OUTBF>
__global__ __launch_bounds__(512, 2) void gemm_bf16_stream_kernel(GemmB16Args g, StreamPlan pl) {
  constexpr int BN = DUAL ? 64 : 128;  // output columns per block
  constexpr int NI = BN / 32;          // 32-column tiles per wave
  constexpr int NOPS = DUAL ? 2 : 1;
  constexpr int PITCH = KP + 8;        // bf16 per LDS row
  constexpr int KS = KP / 16, CPT = 4, CK = KS / CPT;
  static_assert(KS % CPT == 0, "k-steps must split into 4 chunks");
  __shared__ __attribute__((aligned(16))) bfr_t sB[NOPS * BN * PITCH];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int per_xcd = gridDim.x / 8;
  const int x = blockIdx.x % 8, l = blockIdx.x / 8;
  if (l >= pl.groups_per_xcd * pl.nslice) return;
  const int sl = l % pl.nslice;
  const int64_t gid = (int64_t)x * pl.groups_per_xcd + l / pl.nslice, NG = 8 * (int64_t)pl.groups_per_xcd;
  (void)per_xcd;
  const int64_t n0 = (int64_t)sl * BN;
  // stage the Bt slice(s): row r of slice op = Bt[n0 + r][0..KP), zero past N and ldb
  constexpr int CPR = KP / 8;  // 16-B chunks per row
  for (int i = threadIdx.x; i < NOPS * BN * CPR; i += 512) {
    const int op = i / (BN * CPR), rem = i % (BN * CPR), r = rem / CPR, c = rem % CPR;
    const bfr_t* Bt = (DUAL && op) ? g.Bt2 : g.Bt;
    const int64_t n = n0 + r, kc = 8 * c;
    u32x4v v = u32x4v{0u, 0u, 0u, 0u};
    if (n < g.N && kc < g.ldb) v = *reinterpret_cast<const u32x4v*>(Bt + n * g.ldb + kc);
    *reinterpret_cast<u32x4v*>(sB + (op * BN + r) * PITCH + kc) = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int64_t ntiles = (g.M + 255) / 256;  // 256 rows per block step: 8 waves x 32
  if (gid >= ntiles) return;
  const int64_t my_tiles = (ntiles - 1 - gid) / NG + 1;
  const int64_t last = g.M - 1;
  // Chunk c of a tile: operand op = c / CPT (A, then A2 for the dual product -- all of
  // A.Bt's k-steps before A2.Bt2's, the tiled kernel's accumulation order), k-steps
  // (c % CPT) * CK .. + CK.  Fragments of row j of the wave's 32, k 16 ks + 8h.
  constexpr int NCH = CPT * NOPS;
  auto load = [&](int64_t t, int c, bf16x8 (&a)[CK]) {
    const int64_t rr = (gid + t * NG) * 256 + 32 * wave + j;
    const int64_t row = rr < last ? rr : last;
    const bfr_t* A = (DUAL && c >= CPT) ? g.A2 : g.A;
    const int cc = c % CPT;
#pragma unroll
    for (int i = 0; i < CK; ++i) {
      const int64_t kc = 16 * (cc * CK + i) + 8 * h;
      if (cc * CK + i < KS - 1 || kc < g.lda) a[i] = *reinterpret_cast<const bf16x8*>(A + row * g.lda + kc);
      else a[i] = bf16x8{};
    }
  };
  f32x16 acc[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) acc[ni] = zero16();
  auto compute = [&](int c, const bf16x8 (&a)[CK]) {
    const bfr_t* Bs = sB + (c / CPT) * BN * PITCH;
    const int cc = c % CPT;
#pragma unroll
    for (int i = 0; i < CK; ++i) {
      const int ks = cc * CK + i;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(Bs + (32 * ni + j) * PITCH + 16 * ks + 8 * h);
        acc[ni] = MFMA32B(bv, a[i], acc[ni]);
      }
    }
  };
  bf16x8 b0[CK], b1[CK];
  load(0, 0, b0);
  const bool vec = (g.ldc & 3) == 0 && (g.epi != MRL_GEMM_DTANH || (g.ldh & 3) == 0);
  for (int64_t t = 0; t < my_tiles; ++t) {
    const int64_t tn = t + 1 < my_tiles ? t + 1 : t;  // the last tile re-loads itself (unused)
#pragma unroll
    for (int c = 0; c < NCH; c += 2) {
      // the fences keep the scheduler from hoisting later chunks' loads and LDS reads
      // (all of them live at once spilled the whole register file)
      load(t, c + 1, b1);
      compute(c, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (c + 2 < NCH) load(t, c + 2, b0);
      else load(tn, 0, b0);
      compute(c + 1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue of the wave's 32 rows
    const int64_t row = (gid + t * NG) * 256 + 32 * wave + j;
    if (row < g.M) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int64_t cbase = n0 + 32 * ni;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t cc = cbase + 8 * q + 4 * h;
          if (vec && cc + 4 <= g.N) {
            const float4 bb = g.bias != nullptr ? *reinterpret_cast<const float4*>(g.bias + cc)
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
            float v[4] = {acc[ni][4 * q + 0] + bb.x, acc[ni][4 * q + 1] + bb.y, acc[ni][4 * q + 2] + bb.z,
                          acc[ni][4 * q + 3] + bb.w};
            if (g.epi == MRL_GEMM_TANH) {
#pragma unroll
              for (int e = 0; e < 4; e += 2) {
                const f32x2 tt = tanh_fast2(f32x2{v[e], v[e + 1]});
                v[e] = tt.x;
                v[e + 1] = tt.y;
              }
            } else if (g.epi == MRL_GEMM_DTANH) {
              const uint2 hb = *reinterpret_cast<const uint2*>(g.H + row * g.ldh + cc);
              v[0] *= dtanh(__uint_as_float(hb.x << 16));
              v[1] *= dtanh(__uint_as_float(hb.x & 0xffff0000u));
              v[2] *= dtanh(__uint_as_float(hb.y << 16));
              v[3] *= dtanh(__uint_as_float(hb.y & 0xffff0000u));
            }
            if (OUTBF) {
              const uint2 o = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                               (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
              *reinterpret_cast<uint2*>(reinterpret_cast<bfr_t*>(g.C) + row * g.ldc + cc) = o;
            } else {
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + row * g.ldc + cc) =
                  make_float4(v[0], v[1], v[2], v[3]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int64_t col = cc + e;
              if (col >= g.N) continue;
              float xv = acc[ni][4 * q + e] + (g.bias != nullptr ? g.bias[col] : 0.f);
              if (g.epi == MRL_GEMM_TANH) xv = tanh_fast(xv);
              else if (g.epi == MRL_GEMM_DTANH) xv *= dtanh(bf2f(g.H[row * g.ldh + col]));
              if (OUTBF) reinterpret_cast<bfr_t*>(g.C)[row * g.ldc + col] = f2bf(xv);
              else reinterpret_cast<float*>(g.C)[row * g.ldc + col] = xv;
            }
          }
        }
      }
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = zero16();
  }
}

// ------------------------------------------------------------------ 256 x 256 NN GEMM
// The tall layered-path products (M ~ 1 M rows, K <= 512, N = 512) are bound by how many
// operand bytes reach the CU per MFMA: a 128 x 128 tile needs 2 B x 2048 MACs x (1/128 +
// 1/128) = 64 B per CU cycle from L2 at full MFMA rate, a 256 x 256 tile 32 B (L2 serves
// about 30: MI355X_MICROARCH.md, indexed rows).  So: 256 x 256 tiles, 8 waves (2 per SIMD,
// 64 x 128 each, 128 accumulator registers), K staged 32 at a time by LDS-DMA
// (global_load_lds_dwordx4: no staging registers, no ds_write pass) into four 32 KB
// stages, three in flight ahead of the one being read (an L2 / HBM fetch outlasts one
// stage's MFMAs): a counted vmcnt and a raw barrier per stage (a __syncthreads would
// wait for every DMA in flight), the four stages separate LDS objects so the compiler's
// wait for an LDS-DMA in flight is not put in front of another stage's fragment reads.
// Rows of a stage image are 64 B (32 k of one row of A or Bt); the 16-B chunk c of row r
// sits at position c ^ ((r >> 2) & 3) -- applied on the DMA source side, the destination
// being lane-linear -- so a 16-lane ds_read_b128 group (rows r..r+15, one chunk) covers
// the 64 banks once.  Chunks past K read a zero block.  Persistent blocks walk the tiles
// as one stream of stages (the next tile's first stages load under this tile's last
// stages and epilogue); the ntn column tiles of a row block run on blocks of one XCD at
// the same time (A from HBM once, from that XCD's L2 for the others).  Same operands and
// the same per-output k order as gemm_bf16_kernel (k-steps of 16 in order, A.Bt before
// A2.Bt2): bit-identical results.
__device__ const uint32_t kZero16[4] = {0u, 0u, 0u, 0u};
constexpr int BBM = 256, BBN = 256, BBK = 32;
constexpr int BSTAGE = (BBM + BBN) * BBK;  // bf16 per stage: A rows, then Bt rows (16 K each)

struct BigPlan {
  int64_t ntm;  // row tiles
  int ntn;      // column tiles
  int per_xcd;  // blocks per XCD
};

__device__ inline void glds16b(const void* g, bfr_t* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// DT: the DTANH epilogue (H operand), compiled apart so the others carry no H registers
template <bool DUAL, bool OUTBF, bool DT>
__global__ __launch_bounds__(512, 2) void gemm_bf16_big_kernel(GemmB16Args g, BigPlan pl) {
  __shared__ __attribute__((aligned(16))) bfr_t sb0[BSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb1[BSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb2[BSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb3[BSTAGE];
  // the block's bias columns (its column tile is fixed): an epilogue read from LDS, not a
  // global load, whose wait would drain every DMA and store in flight (vmcnt is in order)
  __shared__ __attribute__((aligned(16))) float sbias[BBN];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 rows x 128 columns
  const int xcd = blockIdx.x % 8, y = blockIdx.x / 8;
  if (y >= pl.per_xcd) return;
  const int tn = y % pl.ntn, lr = y / pl.ntn, rows_per_round = pl.per_xcd / pl.ntn;
  if (threadIdx.x < BBN) {
    const int64_t c = (int64_t)tn * BBN + threadIdx.x;
    sbias[threadIdx.x] = (g.bias != nullptr && c < g.N) ? g.bias[c] : 0.f;
  }
  const int64_t tstride = 8 * (int64_t)rows_per_round;
  const int64_t ntk = (g.K + BBK - 1) / BBK, nst = (DUAL ? 2 : 1) * ntk;
  // DMA of stage s of row tile tm into `dst`: waves 0..3 fetch A rows 64 w .. + 63, waves
  // 4..7 Bt rows 64 (w - 4) .. + 63; instruction i covers 16 rows (lane: row L >> 2,
  // position L & 3, i.e. chunk (L & 3) ^ ((row >> 2) & 3) = (L & 3) ^ (L >> 4))
  const bool isA = wave < 4;
  const int lrow = 64 * (wave & 3) + (lane >> 2);
  const int coff = 8 * ((lane & 3) ^ (lane >> 4));
  auto issue = [&](bfr_t* dst, int64_t tm, int64_t s) {
    const bool second = DUAL && s >= ntk;
    const int64_t k0 = (second ? s - ntk : s) * BBK;
    const bfr_t* base = isA ? (second ? g.A2 : g.A) : (second ? g.Bt2 : g.Bt);
    const int64_t ld = isA ? g.lda : g.ldb, lim = isA ? g.M : g.N;
    const int64_t r0 = isA ? tm * BBM : (int64_t)tn * BBN;
    bfr_t* d0 = dst + (isA ? 0 : BBM * BBK) + 64 * (wave & 3) * BBK;
    if (r0 + BBM <= lim && k0 + BBK <= g.K) {
      // interior: a wave-uniform base per instruction and a 32-bit lane offset
      const bfr_t* tb = base + (r0 + 64 * (wave & 3)) * ld + k0;
      const uint32_t lo = (uint32_t)((lane >> 2) * ld + coff);
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16b(tb + 16 * i * ld + lo, d0 + 16 * i * BBK);
    } else {
      // a tile crossing M / N (rows clamped: their outputs are not stored) or the K tail
      // (chunks past K read the zero block)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t k = k0 + coff;
        int64_t row = r0 + lrow + 16 * i;
        row = row < lim ? row : lim - 1;
        const void* src = k < g.K ? (const void*)(base + row * ld + k) : (const void*)kZero16;
        glds16b(src, d0 + 16 * i * BBK);
      }
    }
  };
  // the stage stream: (row tile itm, stage is) is the next stage to load
  int64_t itm = (int64_t)xcd * rows_per_round + lr, is = 0;
  int issued = 0, consumed = 0;
  auto issue_next = [&](bfr_t* dst) {
    if (itm < pl.ntm) {
      issue(dst, itm, is);
      ++issued;
      if (++is == nst) {
        is = 0;
        itm += tstride;
      }
    }
  };
  f32x16 acc[2][4];
  // fragments of one 16-deep k-step: A rows of the wave's two 32-row tiles, Bt rows of its
  // four 32-column tiles (chunk 2 ks + h of each row)
  // The fragment reads are inline asm: the compiler, which tracks only a few LDS-DMAs
  // per object, otherwise drains every DMA and epilogue store in flight (vmcnt 0) in
  // front of the first reads of a tile.  Their completion is the stage's explicit
  // lgkmcnt waits, which take the fragments as operands (no MFMA moves above them).
  struct Frag {
    u32x4v a[2], b[4];
  };
  // lane byte offsets of k-step ks's first A / Bt fragment; the other 32-row tiles sit
  // 2048 B apart with the same swizzle ((r >> 2) & 3 does not see the 32-row step)
  uint32_t offA[2], offB[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c = (2 * ks + h) ^ ((j >> 2) & 3);
    offA[ks] = 2 * ((64 * wm + j) * BBK + 8 * c);
    offB[ks] = 2 * ((BBM + 128 * wn + j) * BBK + 8 * c);
  }
  auto read = [&](const bfr_t* cur, int ks, Frag& f) {
    const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(cur);
    const uint32_t va = base + offA[ks], vb = base + offB[ks];
    asm volatile("ds_read_b128 %0, %1" : "=v"(f.a[0]) : "v"(va));
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(f.a[1]) : "v"(va));
    asm volatile("ds_read_b128 %0, %1" : "=v"(f.b[0]) : "v"(vb));
    asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(f.b[1]) : "v"(vb));
    asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(f.b[2]) : "v"(vb));
    asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(f.b[3]) : "v"(vb));
  };
  auto mfma = [&](const Frag& f) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)  // C^T tiles
        acc[mi][ni] = MFMA32B(__builtin_bit_cast(bf16x8, f.b[ni]), __builtin_bit_cast(bf16x8, f.a[mi]), acc[mi][ni]);
  };
#define MRL_FRAG_OPS(f) "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.b[0]), "+v"(f.b[1]), "+v"(f.b[2]), "+v"(f.b[3])
  // One stage (two k-steps).  Its first k-step's fragments are already in f0 (read under
  // the previous stage); the barrier here certifies the NEXT stage's DMA has landed for
  // every wave (at most the stage after it still in flight) and that every wave is done
  // with the stage loaded next; then that DMA goes out, and the fragment reads of the
  // second k-step and of the next stage's first k-step run under the MFMAs.
  Frag f0, f1;
  // vmcnt retires in issue order and counts stores too: the epilogue's stores of an
  // interior tile (16 per wave with bf16 output, 32 with f32) are issued after the loads
  // of the next tile's first two stages, so those two stages' waits let them stay in
  // flight (vmcnt 4 + stores) instead of draining them.
  int post = 0;
  auto stage = [&](const bfr_t* cur, const bfr_t* next, bfr_t* load) {
    const int later = issued - consumed - 2;  // stages issued after the next one
    if (later >= 1 && post > 0) {
      if (OUTBF) asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" : MRL_FRAG_OPS(f0)::"memory");
      else asm volatile("s_waitcnt vmcnt(36) lgkmcnt(0)" : MRL_FRAG_OPS(f0)::"memory");
    } else if (later >= 1) {
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" : MRL_FRAG_OPS(f0)::"memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : MRL_FRAG_OPS(f0)::"memory");
    }
    post = post > 0 ? post - 1 : 0;
    __builtin_amdgcn_s_barrier();
    // the f0 MFMAs go first (their fragments are in registers), the DMA and the second
    // k-step's reads under them; the next stage's first reads are unconditional (past
    // the stream's end they read a stale stage, unused)
    read(cur, 1, f1);
    mfma(f0);
    issue_next(load);
    read(next, 0, f0);
    asm volatile("s_waitcnt lgkmcnt(6)" : MRL_FRAG_OPS(f1)::"memory");  // f1 (f0's six still in flight)
    mfma(f1);
    ++consumed;
  };
  // 16-B vector epilogue (ldc, ldh multiples of 8)
  const bool vec = (g.ldc & 7) == 0 && (g.epi != MRL_GEMM_DTANH || (g.ldh & 7) == 0);
  __syncthreads();  // sbias
  issue_next(sb0);
  issue_next(sb1);
  issue_next(sb2);
  if (issued > 0) {  // the first stage's first k-step (once per block: wait for all three)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    read(sb0, 0, f0);
  }
  const bool ncols_full = (int64_t)(tn + 1) * BBN <= g.N;
  for (int64_t tm = (int64_t)xcd * rows_per_round + lr; tm < pl.ntm; tm += tstride) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = zero16();
    for (int64_t s = 0; s < nst; s += 4) {  // nst % 4 == 0 (host check): stage s in sb0
      stage(sb0, sb1, sb3);
      stage(sb1, sb2, sb0);
      stage(sb2, sb3, sb1);
      stage(sb3, sb0, sb2);
    }
    // epilogue: lane (j, h) holds row j of each 32 x 32 C tile at columns cperm(r, h) --
    // four runs of 4 consecutive columns, 8q + 4h.  One v_permlane32_swap per register
    // pair (runs q = 2p and 2p + 1) leaves lane (j, h) with the 8 consecutive columns
    // 16p + 8h .. + 7: half the store instructions, 16-B bf16 stores (the epilogue is
    // store-issue-bound: 8-B stores ran 1.1-1.2 x slower).  The next tile's first stages
    // are already in flight.
#ifdef MRL_BIG_ABL_NOEPI  // diagnostic timing build only (tools/build_ablate.sh): no epilogue
    {
      float sacc = 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc += acc[mi][ni][r];
      if (sacc == 1234.5f) reinterpret_cast<float*>(g.C)[tm] = sacc;
      continue;
    }
#endif
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int64_t row = tm * BBM + 64 * wm + 32 * mi + j;
      // DTANH: the H chunks of the 32-row tile issued together (one wait, not eight)
      uint4 hv[DT ? 4 : 1][2];
#pragma unroll
      for (int ni = 0; ni < (DT ? 4 : 1); ++ni)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int64_t c0 = (int64_t)tn * BBN + 128 * wn + 32 * ni + 16 * pp + 8 * h;
          hv[ni][pp] = (DT && vec && row < g.M && c0 + 8 <= g.N)
                           ? *reinterpret_cast<const uint4*>(g.H + row * g.ldh + c0)
                           : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int64_t cbase = (int64_t)tn * BBN + 128 * wn + 32 * ni;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[mi][ni][8 * pp + e]),
                                                             __float_as_uint(acc[mi][ni][8 * pp + 4 + e]), false, false);
            v[e] = __uint_as_float(sw[0]);
            v[4 + e] = __uint_as_float(sw[1]);
          }
          if (row >= g.M) continue;
          const int64_t c0 = cbase + 16 * pp + 8 * h;
          if (vec && c0 + 8 <= g.N) {
            if (g.bias != nullptr) {
              const float* bp = sbias + 128 * wn + 32 * ni + 16 * pp + 8 * h;
              const float4 b0 = *reinterpret_cast<const float4*>(bp);
              const float4 b1 = *reinterpret_cast<const float4*>(bp + 4);
              v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
              v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
            }
            if (!DT && g.epi == MRL_GEMM_TANH) {
#pragma unroll
              for (int e = 0; e < 8; e += 2) {
                const f32x2 t = tanh_fast2(f32x2{v[e], v[e + 1]});
                v[e] = t.x;
                v[e + 1] = t.y;
              }
            } else if (DT) {
              const uint4 hb = hv[DT ? ni : 0][pp];
              const uint32_t hw[4] = {hb.x, hb.y, hb.z, hb.w};
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v[2 * e] *= dtanh(__uint_as_float(hw[e] << 16));
                v[2 * e + 1] *= dtanh(__uint_as_float(hw[e] & 0xffff0000u));
              }
            }
            if (OUTBF) {
              uint4 o;
              o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
              o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
              o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
              o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
              *reinterpret_cast<uint4*>(reinterpret_cast<bfr_t*>(g.C) + row * g.ldc + c0) = o;
            } else {
              float* cp = reinterpret_cast<float*>(g.C) + row * g.ldc + c0;
              *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
              *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
            continue;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int64_t col = c0 + e;
            if (col >= g.N) continue;
            float xv = v[e] + (g.bias != nullptr ? g.bias[col] : 0.f);
            if (!DT && g.epi == MRL_GEMM_TANH) xv = tanh_fast(xv);
            else if (DT) xv *= dtanh(bf2f(g.H[row * g.ldh + col]));
            if (OUTBF) reinterpret_cast<bfr_t*>(g.C)[row * g.ldc + col] = f2bf(xv);
            else reinterpret_cast<float*>(g.C)[row * g.ldc + col] = xv;
          }
        }
      }
    }
    // every lane of an interior tile issued all its vector stores (the count above)
    post = (vec && ncols_full && (tm + 1) * BBM <= g.M) ? 2 : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the block
}

// ------------------------------------------------------------------ small-M NN GEMM
// The Humanoid rollout's per-step hidden layers (M = E = 1024 rows, K <= 512, N = 512)
// are latency-bound: the 128 x 128 tiled kernel gives 32 blocks a serial 8-stage K loop.
// Here a block takes a 64 x 64 tile (four waves of 32 x 32, one accumulator each) and
// stages its whole A / Bt panels (K <= 512) by LDS-DMA at entry, as four K quarters
// (128 k each) in separate LDS objects: quarter q's MFMAs start as soon as its DMA has
// landed (counted vmcnt + barrier) while the later quarters are still in flight.  Image
// [row][16 chunks] per quarter (256-B rows), chunk c of row r at c ^ (r & 15): the 16
// rows of a ds_read_b128 lane group cover the 64 banks once.  Same k order per output
// as gemm_bf16_kernel (k-steps of 16 ascending): bit-identical results.
constexpr int SBM = 64, SBN = 64, SQK = 128;  // tile, K per quarter
constexpr int SQ_ELEMS = SBM * SQK;            // bf16 per quarter image (16 KB)

template <bool OUTBF>
__global__ __launch_bounds__(256) void gemm_bf16_small_kernel(GemmB16Args g) {
  __shared__ __attribute__((aligned(16))) bfr_t a0[SQ_ELEMS], a1[SQ_ELEMS], a2[SQ_ELEMS], a3[SQ_ELEMS];
  __shared__ __attribute__((aligned(16))) bfr_t b0[SQ_ELEMS], b1[SQ_ELEMS], b2[SQ_ELEMS], b3[SQ_ELEMS];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * SBM, n0 = (int64_t)blockIdx.x * SBN;
  const int nq = (int)((g.K + SQK - 1) / SQK);  // quarters (host: K <= 512); k past K reads zeros
  // DMA: wave w, instruction i covers rows 16 w + 4 i + (lane >> 4), position lane & 15
  const int pos = lane & 15;
  auto dma = [&](bfr_t* qa, bfr_t* qb, int q) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * wave + 4 * i + (lane >> 4);
      const int c = pos ^ (r & 15);
      const int64_t k = (int64_t)q * SQK + 8 * c;
      const int64_t ra = min(m0 + r, g.M - 1), rb = min(n0 + r, g.N - 1);
      const void* sa = k < g.K ? (const void*)(g.A + ra * g.lda + k) : (const void*)kZero16;
      const void* sb = k < g.K ? (const void*)(g.Bt + rb * g.ldb + k) : (const void*)kZero16;
      glds16b(sa, qa + (16 * wave + 4 * i) * 128);
      glds16b(sb, qb + (16 * wave + 4 * i) * 128);
    }
  };
  dma(a0, b0, 0);
  if (nq > 1) dma(a1, b1, 1);
  if (nq > 2) dma(a2, b2, 2);
  if (nq > 3) dma(a3, b3, 3);
  f32x16 acc = zero16();
  const int ra = 32 * wm + j, rb = 32 * wn + j;
  // quarter q: this wave's DMA of it has landed (8 instructions per later quarter still
  // in flight), then every wave's (the barrier); 8 k-steps, branch-free (zeros past K)
  auto quarter = [&](const bfr_t* As, const bfr_t* Bs, int later) {
    if (later >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (later == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the fragment reads as inline asm: the compiler's LDS-DMA alias tracking (a few
    // DMAs deep) would otherwise drain every quarter still in flight (vmcnt 0) before
    // them; their completion is this lambda's explicit lgkmcnt wait, which takes the
    // fragments as operands so no MFMA is scheduled above it
    u32x4v av[8], bv[8];
    const uint32_t la = (uint32_t)reinterpret_cast<uintptr_t>(As) + 2 * ra * 128;
    const uint32_t lb = (uint32_t)reinterpret_cast<uintptr_t>(Bs) + 2 * rb * 128;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int c = 2 * ks + h;
      asm volatile("ds_read_b128 %0, %1" : "=v"(av[ks]) : "v"(la + 16 * (c ^ (ra & 15))));
      asm volatile("ds_read_b128 %0, %1" : "=v"(bv[ks]) : "v"(lb + 16 * (c ^ (rb & 15))));
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]), "+v"(av[4]), "+v"(av[5]), "+v"(av[6]),
                   "+v"(av[7]), "+v"(bv[0]), "+v"(bv[1]), "+v"(bv[2]), "+v"(bv[3]), "+v"(bv[4]), "+v"(bv[5]),
                   "+v"(bv[6]), "+v"(bv[7]));
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)  // C^T tile: lane (j, h) holds row j
      acc = MFMA32B(__builtin_bit_cast(bf16x8, bv[ks]), __builtin_bit_cast(bf16x8, av[ks]), acc);
  };
  quarter(a0, b0, nq - 1);
  if (nq > 1) quarter(a1, b1, nq - 2);
  if (nq > 2) quarter(a2, b2, nq - 3);
  if (nq > 3) quarter(a3, b3, 0);
  // epilogue (gemm_bf16_kernel's, one 32 x 32 tile per wave)
  const int64_t row = m0 + 32 * wm + j;
  if (row >= g.M) return;
  const bool vec = (g.ldc & 3) == 0;
  const int64_t cbase = n0 + 32 * wn;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t c0 = cbase + 8 * q + 4 * h;
    float v[4];
    if (vec && c0 + 4 <= g.N) {
      const float4 b = g.bias != nullptr ? *reinterpret_cast<const float4*>(g.bias + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[0] = acc[4 * q + 0] + b.x;
      v[1] = acc[4 * q + 1] + b.y;
      v[2] = acc[4 * q + 2] + b.z;
      v[3] = acc[4 * q + 3] + b.w;
      if (g.epi == MRL_GEMM_TANH) {
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 t = tanh_fast2(f32x2{v[e], v[e + 1]});
          v[e] = t.x;
          v[e + 1] = t.y;
        }
      }
      if (OUTBF) {
        const uint2 o = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                         (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
        *reinterpret_cast<uint2*>(reinterpret_cast<bfr_t*>(g.C) + row * g.ldc + c0) = o;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + row * g.ldc + c0) = make_float4(v[0], v[1], v[2], v[3]);
      }
      continue;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t col = c0 + e;
      if (col >= g.N) continue;
      float x = acc[4 * q + e] + (g.bias != nullptr ? g.bias[col] : 0.f);
      if (g.epi == MRL_GEMM_TANH) x = tanh_fast(x);
      if (OUTBF) reinterpret_cast<bfr_t*>(g.C)[row * g.ldc + col] = f2bf(x);
      else reinterpret_cast<float*>(g.C)[row * g.ldc + col] = x;
    }
  }
}

// ------------------------------------------------------------------ TN (weight grads)
// K step: 32 rows; LDS images [32 rows][BM or BN columns], pitch 160 bf16 (320 B): a
// 32-lane half's transposed read (rows q = 0..3, 8 B at columns 16G + 4p) covers all
// 64 banks once.
constexpr int TBK = 32, TLD = 160;

struct GemmTnArgs {
  int64_t M, N, K;  // C[M][N] over K rows
  const bfr_t* A;   // [K][lda]: columns 0..m_real-1 (column m_real = 1 if ones)
  const bfr_t* B;   // [K][ldb]
  int64_t lda, ldb;
  int64_t m_real;
  int64_t k_chunk;  // rows per split
  float* slab;
  int64_t slab_stride, ldc;
  const int32_t* skip;
};

// the 8 columns c0 .. c0+7 of row r as a 16-B chunk; column m_real reads as 1 (the
// ones-column of the bias gradient), columns past it as 0
__device__ inline u32x4v load_row_chunk(const bfr_t* __restrict__ p, int64_t r, int64_t r_end, int64_t ld,
                                        int64_t c0, int64_t creal, int64_t cmax, bool ones) {
  if (r >= r_end) return u32x4v{0u, 0u, 0u, 0u};
  if (c0 + 8 <= creal) return *reinterpret_cast<const u32x4v*>(p + r * ld + c0);
  uint16_t v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int64_t c = c0 + q;
    v[q] = c < creal ? p[r * ld + c] : ((ones && c == creal && c < cmax) ? (uint16_t)0x3F80 : (uint16_t)0);
  }
  return u32x4v{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
}

// 8 consecutive k (rows 8kg .. 8kg+7 of the 16-row k step `ks`) of column
// c0 + (lane & 31) from a [rows][TLD] image: two transposing reads of 4 rows each
__device__ inline bf16x8 tr_operand(const bfr_t* img, int c0, int ks, int lane) {
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;  // lane 4q + p: row q, columns 4p .. 4p+3
  const int kg = G >> 1, col = c0 + 16 * (G & 1) + 4 * p;
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  const bfr_t* r0 = img + (16 * ks + 8 * kg + q) * TLD + col;
  // (the v4bf16 form and one shuffle: element-wise bit casts of the i16 form were
  // lowered to permutes that duplicated elements)
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(r0));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(r0 + 4 * TLD));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int BN>
__global__ __launch_bounds__(256) void gemm_bf16_tn_kernel(GemmTnArgs g) {
  constexpr int MI = BN == 128 ? 2 : 1, NI = MI;
  constexpr int NA = TBK * (QBM / 8) / 256, NB = TBK * (BN / 8) / 256 > 0 ? TBK * (BN / 8) / 256 : 1;
  constexpr int STAGE = 2 * TBK * TLD;  // A image then B image
  __shared__ __attribute__((aligned(16))) bfr_t smem[2 * STAGE];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int wm = BN == 128 ? wave >> 1 : wave, wn = BN == 128 ? wave & 1 : 0;
  const int64_t m0 = (int64_t)blockIdx.y * QBM, n0 = (int64_t)blockIdx.x * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * g.k_chunk, kend = min(g.K, kbeg + g.k_chunk);
  const int64_t nt = kend > kbeg ? (kend - kbeg + TBK - 1) / TBK : 0;
  // A rows: thread t stages 16-B chunk t & 15 (columns 8c) of rows t >> 4 (+ 16 i);
  // B (BN = 128) the same; B (BN = 32): chunk t & 3 of row t >> 2 (threads < 128)
  const int ac = threadIdx.x & 15, ar = threadIdx.x >> 4;
  const int bcw = BN / 8, bc = threadIdx.x % bcw, br = threadIdx.x / bcw;
  const bool b_active = threadIdx.x < TBK * bcw;
  u32x4v ra[NA], rb[NB];
  auto load = [&](int64_t t) {
    const int64_t k0 = kbeg + t * TBK;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      ra[i] = load_row_chunk(g.A, k0 + ar + 16 * i, kend, g.lda, m0 + 8 * ac, g.m_real, g.M, g.M > g.m_real);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = b_active ? load_row_chunk(g.B, k0 + br + (256 / bcw) * i, kend, g.ldb, n0 + 8 * bc, g.N, g.N, false)
                       : u32x4v{0u, 0u, 0u, 0u};
  };
  auto store = [&](bfr_t* st) {
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<u32x4v*>(st + (ar + 16 * i) * TLD + 8 * ac) = ra[i];
    if (b_active)
#pragma unroll
      for (int i = 0; i < NB; ++i)
        *reinterpret_cast<u32x4v*>(st + TBK * TLD + (br + (256 / bcw) * i) * TLD + 8 * bc) = rb[i];
  };
  f32x16 acc[MI][NI];
#pragma unroll
  for (int a = 0; a < MI; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b) acc[a][b] = zero16();
  if (nt > 0) {
    load(0);
    store(smem);
  }
  for (int64_t t = 0; t < nt; ++t) {
    __syncthreads();
    const bfr_t* As = smem + (t & 1) * STAGE;
    const bfr_t* Bs = As + TBK * TLD;
    if (t + 1 < nt) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < TBK / 16; ++ks) {
      bf16x8 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) av[mi] = tr_operand(As, wm * 32 * MI + 32 * mi, ks, lane);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bv[ni] = tr_operand(Bs, wn * 32 * NI + 32 * ni, ks, lane);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA32B(av[mi], bv[ni], acc[mi][ni]);
    }
    if (t + 1 < nt) store(smem + ((t + 1) & 1) * STAGE);
  }
  float* C = g.slab + (int64_t)blockIdx.z * g.slab_stride;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int64_t col = n0 + wn * 32 * NI + ni * 32 + j;
      if (col >= g.N) continue;
      const int64_t rbase = m0 + wm * 32 * MI + mi * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + cperm(r, h);
        if (row < g.M) C[row * g.ldc + col] = acc[mi][ni][r];
      }
    }
}

// ------------------------------------------------------------------ TN on 256 x 256 tiles
// The layered VJP's weight gradients at Humanoid scale (C = A^T B over K = 1 M rows,
// M = N = 512, 64 split-K slabs): the 128 x 128 kernel above re-reads each operand row
// four times through L2 and stages through registers.  Here a block owns one 256 x 256
// tile of one slab: 8 waves (4 x 2, 64 x 128 each), 32-row stages of A and B (512-B
// image rows, 16 KB each) filled by LDS-DMA, four stage buffers with three in flight
// (the NN big kernel's counted-vmcnt / raw-barrier stream), transposed MFMA operands by
// ds_read_b64_tr_b16.  Chunk c of image row R sits at position c ^ ((R & 3) << 2): the
// four rows of a transposing read's 32-lane half land on distinct 64-B bank segments.
// The four tiles of a slab run on one XCD (A and B chunk rows from HBM once).  Reads are
// inline asm (the compiler's LDS-DMA alias tracking would drain the DMA in flight).
// Same per-slab k order as gemm_bf16_tn_kernel: bit-identical slabs.  The ones-row of
// the bias gradient (ONES) is not a mostly-empty third tile: the blocks of row tile 0
// issue one more (16 x 16 x 32) MFMA per k-step on their B fragment of column group wm
// (the eight waves cover the 256 columns), read as a 16 x 16 x 32 operand: a 0 / 1
// selector A makes its output rows 0 and 1 the column sums of columns 0-15 and 16-31.
constexpr int TBM = 256, TBN = 256, TSK = 32;  // tile, rows per stage
constexpr int TSTAGE = (TBM + TBN) * TSK;      // bf16 per stage (A image, then B)
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

struct TnPlan {
  int ntm, ntn, nsplit;
};

template <bool ONES>
__global__ __launch_bounds__(512, 2) void gemm_bf16_tn_big_kernel(GemmTnArgs g, TnPlan pl) {
  __shared__ __attribute__((aligned(16))) bfr_t sb0[TSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb1[TSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb2[TSTAGE];
  __shared__ __attribute__((aligned(16))) bfr_t sb3[TSTAGE];
  if (g.skip != nullptr && *g.skip != 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // block -> (slab z, tile): the tiles of a slab on one XCD
  const int ntile = pl.ntm * pl.ntn;
  const int xcd = blockIdx.x % 8, y = blockIdx.x / 8;
  const int z = xcd + 8 * (y / ntile), tile = y % ntile;
  if (z >= pl.nsplit) return;
  const int tm = tile / pl.ntn, tn = tile % pl.ntn;
  const int64_t m0 = (int64_t)tm * TBM, n0 = (int64_t)tn * TBN;
  const int64_t kbeg = (int64_t)z * g.k_chunk, kend = min(g.K, kbeg + g.k_chunk);
  const int64_t nst = kend > kbeg ? (kend - kbeg + TSK - 1) / TSK : 0;
  // DMA: waves 0..3 the A image, 4..7 the B image; instruction i of wave w covers image
  // rows 8 (w & 3) + 2 i + (lane >> 5), position lane & 31 (chunk pos ^ ((row & 3) << 2))
  const bool isA = wave < 4;
  const int pos = lane & 31;
  auto issue = [&](bfr_t* dst, int64_t st) {
    const bfr_t* base = isA ? g.A : g.B;
    const int64_t ld = isA ? g.lda : g.ldb, cols = isA ? g.m_real : g.N, c0 = isA ? m0 : n0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 8 * (wave & 3) + 2 * i + (lane >> 5);
      const int c = pos ^ ((row & 3) << 2);
      const int64_t r = kbeg + st * TSK + row, col = c0 + 8 * c;
      const void* src = (r < kend && col < cols) ? (const void*)(base + r * ld + col) : (const void*)kZero16;
      glds16b(src, dst + (isA ? 0 : TBM * TSK) + (8 * (wave & 3) + 2 * i) * 256);
    }
  };
  int64_t issued = 0, consumed = 0;
  auto issue_next = [&](bfr_t* dst) {
    if (issued < nst) {
      issue(dst, issued);
      ++issued;
    }
  };
  // transposing reads (tr_operand's lane map): lane (G = lane >> 4, q, p) reads 8 B at
  // row 16 ks + 8 (G >> 1) + q (+ 4: the second read) and column c0 + 16 (G & 1) + 4 p
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto lane_off = [&](int img_col0, int c0) {  // byte offset in the stage of k-step 0's first read
    const int col = c0 + 16 * (G & 1) + 4 * p;
    const int R = 8 * (G >> 1) + q;
    return (uint32_t)(2 * (img_col0 * TSK) + R * 512 + (((col >> 3) ^ (q << 2)) << 4) + ((col & 7) << 1));
  };
  uint32_t offA[2], offB[4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) offA[mi] = lane_off(0, 64 * wm + 32 * mi);
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) offB[ni] = lane_off(TBM, 128 * wn + 32 * ni);
  struct Frag {
    u32x2v a[2][2], b[4][2];  // [tile][lo / hi]
  };
  // k-step ks (0 / 1) of a stage: rows 16 ks .. (8 KB apart), hi = +4 rows (2 KB)
  auto read = [&](const bfr_t* cur, int ks, Frag& f) {
    const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(cur);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const uint32_t v = base + offA[mi];
      if (ks == 0) {
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.a[mi][0]) : "v"(v));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(f.a[mi][1]) : "v"(v));
      } else {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:8192" : "=v"(f.a[mi][0]) : "v"(v));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:10240" : "=v"(f.a[mi][1]) : "v"(v));
      }
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const uint32_t v = base + offB[ni];
      if (ks == 0) {
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.b[ni][0]) : "v"(v));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(f.b[ni][1]) : "v"(v));
      } else {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:8192" : "=v"(f.b[ni][0]) : "v"(v));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:10240" : "=v"(f.b[ni][1]) : "v"(v));
      }
    }
  };
  f32x16 acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = zero16();
  // ONES: the 32-column group wm's B fragment (lane l: column l & 31, k 8 (l >> 5) ..)
  // as a 16x16x32 B operand is column l & 15 at k-group l >> 4, i.e. k-groups 0 / 2 hold
  // columns 0-15 and 1 / 3 columns 16-31; selector rows 0 / 1 sum either pair
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  const bool ones_blk = ONES && tm == 0;
  bf16x8 sel8;
  {
    const int r = lane & 15, kg = lane >> 4;
    const bool on = (r == 0 && (kg & 1) == 0) || (r == 1 && (kg & 1) == 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) sel8[e] = (__bf16)(on ? 1.0f : 0.0f);
  }
  auto op = [](const u32x2v* lohi) {
    const bf16x4 lo = __builtin_bit_cast(bf16x4, lohi[0]);
    const bf16x4 hi = __builtin_bit_cast(bf16x4, lohi[1]);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto mfma = [&](const Frag& f) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = MFMA32B(op(f.a[mi]), op(f.b[ni]), acc[mi][ni]);
    if (ONES && ones_blk) {  // wave-uniform branches: no copies of the fragment
      if (wm == 0) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel8, op(f.b[0]), acc1, 0, 0, 0);
      else if (wm == 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel8, op(f.b[1]), acc1, 0, 0, 0);
      else if (wm == 2) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel8, op(f.b[2]), acc1, 0, 0, 0);
      else acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel8, op(f.b[3]), acc1, 0, 0, 0);
    }
  };
#define MRL_TN_FRAG(f)                                                                                      \
  "+v"(f.a[0][0]), "+v"(f.a[0][1]), "+v"(f.a[1][0]), "+v"(f.a[1][1]), "+v"(f.b[0][0]), "+v"(f.b[0][1]),    \
      "+v"(f.b[1][0]), "+v"(f.b[1][1]), "+v"(f.b[2][0]), "+v"(f.b[2][1]), "+v"(f.b[3][0]), "+v"(f.b[3][1])
  Frag f0, f1;
  // one stage (two k-steps), the NN big kernel's stream: the next stage's DMA has landed
  // for every wave (at most one more in flight), then the stage after next is issued
  auto stage = [&](const bfr_t* cur, const bfr_t* next, bfr_t* load) {
    const int64_t later = issued - consumed - 2;
    if (later >= 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" : MRL_TN_FRAG(f0)::"memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : MRL_TN_FRAG(f0)::"memory");
    __builtin_amdgcn_s_barrier();
    read(cur, 1, f1);
    mfma(f0);
    issue_next(load);
    read(next, 0, f0);
    asm volatile("s_waitcnt lgkmcnt(12)" : MRL_TN_FRAG(f1)::"memory");
    mfma(f1);
    ++consumed;
  };
  issue_next(sb0);
  issue_next(sb1);
  issue_next(sb2);
  if (nst > 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    read(sb0, 0, f0);
  }
  // nst stages in groups of four (sb0..sb3); a tail stage past nst reads a zero-filled
  // image?  No: stages past nst are skipped by the guard, their buffers never read.
  for (int64_t st = 0; st < nst; st += 4) {
    stage(sb0, sb1, sb3);
    if (st + 1 < nst) stage(sb1, sb2, sb0);
    if (st + 2 < nst) stage(sb2, sb3, sb1);
    if (st + 3 < nst) stage(sb3, sb0, sb2);
  }
#undef MRL_TN_FRAG
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // slab tile: lane j holds column n0 + .. + j, rows cperm(r, h) (gemm_bf16_tn_kernel's)
  float* C = g.slab + (int64_t)z * g.slab_stride;
  const int h = lane >> 5, j = lane & 31;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int64_t col = n0 + 128 * wn + 32 * ni + j;
      if (col >= g.N) continue;
      const int64_t rbase = m0 + 64 * wm + 32 * mi;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + cperm(r, h);
        if (row < g.m_real) C[row * g.ldc + col] = acc[mi][ni][r];
      }
    }
  if (ONES && ones_blk && lane < 16) {  // 16x16 output: lane l holds rows 0..3 of column l
    const int64_t col = n0 + 128 * wn + 32 * wm + lane;
    if (col < g.N) C[g.m_real * g.ldc + col] = acc1[0];
    if (col + 16 < g.N) C[g.m_real * g.ldc + col + 16] = acc1[1];
  }
}

// ------------------------------------------------------------------ casts / packs
// y[r][c] = bf16(x[r][c]) for c < cols, 0 for cols <= c < ldy (zero K padding)
__global__ void cast_rows_bf16_kernel(const float* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx,
                                      bfr_t* __restrict__ y, int64_t ldy) {
  const int64_t total = rows * ldy;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ldy, c = i % ldy;
    y[i] = c < cols ? f2bf(x[r * ldx + c]) : (bfr_t)0;
  }
}

// W [din][dout] (f32, row-major) -> bf16 image: transpose 0: [din][ld] (= W, zero
// columns dout..ld-1), transpose 1: [dout][ld] (= W^T, zero columns din..ld-1)
__global__ void pack_w_bf16_kernel(const float* __restrict__ w, int64_t din, int64_t dout, int transpose,
                                   bfr_t* __restrict__ out, int64_t ld) {
  const int64_t rows = transpose ? dout : din, cols = transpose ? din : dout;
  const int64_t total = rows * ld;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ld, c = i % ld;
    out[i] = c < cols ? f2bf(transpose ? w[c * dout + r] : w[r * dout + c]) : (bfr_t)0;
  }
}

}  // namespace mrl

using namespace mrl;

#ifndef MRL_GEMM_STREAM_MIN_M  // rows from which the streaming kernel takes the NN GEMM (0: never)
#define MRL_GEMM_STREAM_MIN_M 32768
#endif
#ifndef MRL_GEMM_SMALL_MAX_M  // rows up to which the whole-K 64 x 64 kernel takes the NN GEMM (0: never)
#define MRL_GEMM_SMALL_MAX_M 8192
#endif
#ifndef MRL_GEMM_BIG_MIN_M  // rows from which the 256 x 256 LDS-DMA kernel takes the NN GEMM (0: never)
#define MRL_GEMM_BIG_MIN_M 65536
#endif
// The 256 x 256 kernel for a tall NN product (a multiple of four 32-deep K stages, N >= 128,
// one 512-thread block per CU): launched here and true, or false.
static bool big_gemm_launch(const GemmB16Args& g, bool outbf, bool dual, hipStream_t s) {
  const char* e = getenv("MRL_GEMM_BIG_MIN_M");
  const int64_t min_m = e ? atoll(e) : MRL_GEMM_BIG_MIN_M;
  const int64_t ntk = (g.K + BBK - 1) / BBK, nst = (dual ? 2 : 1) * ntk;
  if (min_m <= 0 || g.M < min_m || g.N < 128 || nst % 4 != 0) return false;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  if (ncu < 8 || ncu % 8) return false;
  BigPlan pl;
  pl.ntm = (g.M + BBM - 1) / BBM;
  pl.ntn = (int)((g.N + BBN - 1) / BBN);
  pl.per_xcd = (ncu / 8) / pl.ntn * pl.ntn;  // whole groups of the ntn column tiles
  if (pl.per_xcd < pl.ntn) return false;
  const dim3 grid((unsigned)(8 * pl.per_xcd)), blk(512);
#define MRL_BIG(DU, OB)                                                                       \
  do {                                                                                        \
    if (g.epi == MRL_GEMM_DTANH) hipLaunchKernelGGL((gemm_bf16_big_kernel<DU, OB, true>), grid, blk, 0, s, g, pl); \
    else hipLaunchKernelGGL((gemm_bf16_big_kernel<DU, OB, false>), grid, blk, 0, s, g, pl);   \
  } while (0)
  if (dual) { if (outbf) MRL_BIG(true, true); else MRL_BIG(true, false); }
  else { if (outbf) MRL_BIG(false, true); else MRL_BIG(false, false); }
#undef MRL_BIG
  return true;
}

// The streaming kernel for a tall NN product (K of 257..512, N >= 64, one block per CU):
// launched here and true, or false (the tiled kernel runs).
static bool stream_gemm_launch(const GemmB16Args& g, bool outbf, bool dual, hipStream_t s) {
  const int env_min = []() {
    const char* e = getenv("MRL_GEMM_STREAM_MIN_M");
    return e ? atoi(e) : MRL_GEMM_STREAM_MIN_M;
  }();
  // the dual product (JVP: A.B + A2.B2) measured slower streamed (2.72 vs 1.93 ms at
  // M = 1 M, K = N = 512: twice the A traffic per MFMA through one BN = 64 slice) -> tiled
  if (env_min <= 0 || dual || g.M < env_min || g.N < 64 || g.K <= 256 || g.K > 512) return false;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  if (ncu < 8 || ncu % 8) return false;
  const int bn = dual ? 64 : 128;
  StreamPlan pl;
  pl.nslice = (int)((g.N + bn - 1) / bn);
  pl.groups_per_xcd = (ncu / 8) / pl.nslice;
  if (pl.groups_per_xcd < 1) return false;
  const dim3 grid((unsigned)ncu), blk(512);
#define MRL_STREAM(KP, DU, OB) hipLaunchKernelGGL((gemm_bf16_stream_kernel<KP, DU, OB>), grid, blk, 0, s, g, pl)
  if (g.K <= 384) {
    if (outbf) MRL_STREAM(384, false, true); else MRL_STREAM(384, false, false);
  } else {
    if (outbf) MRL_STREAM(512, false, true); else MRL_STREAM(512, false, false);
  }
#undef MRL_STREAM
  return true;
}

extern "C" {

int mrl_gemm_bf16(const mrl_gemm_bf16_desc* d, const int32_t* skip, void* stream) {
  if (!d || !d->a || !d->bt || !d->c) return fail(E_ARG, "mrl_gemm_bf16: null pointer");
  if ((d->a2 == nullptr) != (d->bt2 == nullptr)) return fail(E_ARG, "mrl_gemm_bf16: a2/bt2 must be both set or both null");
  if (d->epilogue < MRL_GEMM_STORE || d->epilogue > MRL_GEMM_DTANH) return fail(E_ARG, "mrl_gemm_bf16: bad epilogue");
  if (d->epilogue == MRL_GEMM_DTANH && !d->h) return fail(E_ARG, "mrl_gemm_bf16: DTANH needs h");
  if ((d->lda & 7) || (d->ldb & 7) || d->lda < d->k || d->ldb < d->k)
    return fail(E_ARG, "mrl_gemm_bf16: lda / ldb must be multiples of 8 and >= k (zero padding columns)");
  const uintptr_t al = reinterpret_cast<uintptr_t>(d->a) | reinterpret_cast<uintptr_t>(d->bt) |
                       reinterpret_cast<uintptr_t>(d->a2) | reinterpret_cast<uintptr_t>(d->bt2);
  if (al & 15) return fail(E_ARG, "mrl_gemm_bf16: operands must be 16-byte aligned");
  if (d->m <= 0 || d->n <= 0) return OK;
  GemmB16Args g;
  g.M = d->m;
  g.N = d->n;
  g.K = d->k;
  g.A = d->a;
  g.Bt = d->bt;
  g.A2 = d->a2;
  g.Bt2 = d->bt2;
  g.lda = d->lda;
  g.ldb = d->ldb;
  g.C = d->c;
  g.ldc = d->ldc;
  g.bias = d->bias;
  g.H = d->h;
  g.ldh = d->ldh;
  g.epi = d->epilogue;
  g.skip = skip;
  hipStream_t s = (hipStream_t)stream;
  const unsigned gm = (unsigned)((g.M + QBM - 1) / QBM);
  const bool bf = d->c_bf16 != 0;
#ifndef MRL_GEMM_BF16_BK
#define MRL_GEMM_BF16_BK 64
#endif
  constexpr int BK = MRL_GEMM_BF16_BK;
  // lds_limit: the tiled kernel only (the big, streaming and small-M kernels hold 100-132 KB
  // of LDS per block, the first two for the whole product), with 32-deep K stages when the
  // 64-deep ones do not fit the limit; every NN kernel sums each output's k-steps of 16 in
  // the same order, so the results do not change
  const int64_t lim = d->lds_limit > 0 ? d->lds_limit : 0;
  if (lim > 0) {
    const bool k64 = (int64_t)sizeof(bfr_t) * 2 * (QBM + (g.N <= 32 ? 32 : 128)) * (64 + 8) <= lim;
#define MRL_TILED(BKX)                                                                                      \
  do {                                                                                                      \
    if (g.N <= 32) {                                                                                        \
      if (bf) hipLaunchKernelGGL((gemm_bf16_kernel<32, true, BKX>), dim3(1, gm), dim3(256), 0, s, g);        \
      else hipLaunchKernelGGL((gemm_bf16_kernel<32, false, BKX>), dim3(1, gm), dim3(256), 0, s, g);          \
    } else {                                                                                                \
      const dim3 grid((unsigned)((g.N + 127) / 128), gm);                                                   \
      if (bf) hipLaunchKernelGGL((gemm_bf16_kernel<128, true, BKX>), grid, dim3(256), 0, s, g);              \
      else hipLaunchKernelGGL((gemm_bf16_kernel<128, false, BKX>), grid, dim3(256), 0, s, g);                \
    }                                                                                                       \
  } while (0)
    if (k64) MRL_TILED(64);
    else MRL_TILED(32);
#undef MRL_TILED
    return hip_check(hipGetLastError(), "mrl_gemm_bf16");
  }
  if (big_gemm_launch(g, bf, d->a2 != nullptr, s)) return hip_check(hipGetLastError(), "mrl_gemm_bf16");
  {
    // small M (the Humanoid rollout's per-step layers): whole-K panels, 64 x 64 tiles
    const char* e = getenv("MRL_GEMM_SMALL_MAX_M");
    const int64_t max_m = e ? atoll(e) : MRL_GEMM_SMALL_MAX_M;
    if (d->a2 == nullptr && g.M <= max_m && g.K <= 4 * SQK && g.N >= 64 && g.epi != MRL_GEMM_DTANH) {
      const dim3 grid((unsigned)((g.N + SBN - 1) / SBN), (unsigned)((g.M + SBM - 1) / SBM));
      if (bf) hipLaunchKernelGGL((gemm_bf16_small_kernel<true>), grid, dim3(256), 0, s, g);
      else hipLaunchKernelGGL((gemm_bf16_small_kernel<false>), grid, dim3(256), 0, s, g);
      return hip_check(hipGetLastError(), "mrl_gemm_bf16");
    }
  }
  if (stream_gemm_launch(g, bf, d->a2 != nullptr, s)) return hip_check(hipGetLastError(), "mrl_gemm_bf16");
  if (g.N <= 32) {
    const dim3 grid(1, gm);
    if (bf) hipLaunchKernelGGL((gemm_bf16_kernel<32, true, BK>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_bf16_kernel<32, false, BK>), grid, dim3(256), 0, s, g);
  } else {
    const dim3 grid((unsigned)((g.N + 127) / 128), gm);
    if (bf) hipLaunchKernelGGL((gemm_bf16_kernel<128, true, BK>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_bf16_kernel<128, false, BK>), grid, dim3(256), 0, s, g);
  }
  return hip_check(hipGetLastError(), "mrl_gemm_bf16");
}

int mrl_gemm_bf16_tn(const mrl_gemm_bf16_tn_desc* d, const int32_t* skip, void* stream) {
  if (!d || !d->a || !d->b || !d->slab) return fail(E_ARG, "mrl_gemm_bf16_tn: null pointer");
  const int64_t m_real = d->m - (d->ones_row ? 1 : 0);
  if ((d->lda & 7) || (d->ldb & 7) || d->lda < m_real || d->ldb < d->n)
    return fail(E_ARG, "mrl_gemm_bf16_tn: lda / ldb must be multiples of 8 covering the columns");
  if ((reinterpret_cast<uintptr_t>(d->a) | reinterpret_cast<uintptr_t>(d->b)) & 15)
    return fail(E_ARG, "mrl_gemm_bf16_tn: operands must be 16-byte aligned");
  if (d->m <= 0 || d->n <= 0) return OK;
  GemmTnArgs g;
  g.M = d->m;
  g.N = d->n;
  g.K = d->k;
  g.A = d->a;
  g.B = d->b;
  g.lda = d->lda;
  g.ldb = d->ldb;
  g.m_real = m_real;
  // the split of gemm.hip's slab GEMMs (mrl_gemm_slab_splits slabs of whole 32-row steps)
  const int64_t req = d->splits < 1 ? 1 : d->splits;
  g.k_chunk = ((d->k + req - 1) / req + TBK - 1) / TBK * TBK;
  if (g.k_chunk < TBK) g.k_chunk = TBK;
  const int64_t z = d->k > 0 ? (d->k + g.k_chunk - 1) / g.k_chunk : 1;
  if (z > 65535) return fail(E_ARG, "mrl_gemm_bf16_tn: too many splits");
  g.slab = d->slab;
  g.slab_stride = d->slab_stride;
  g.ldc = d->ldc;
  g.skip = skip;
  hipStream_t s = (hipStream_t)stream;
  {
    // 256 x 256 tiles for the wide layers (m_real, N >= 256; the ones-row rides row tile 0)
    const char* e = getenv("MRL_GEMM_TN_BIG");
    const bool big = (e ? atoi(e) != 0 : true) && d->lds_limit <= 0;  // lds_limit: the 41 KB tiled kernel
    if (big && g.m_real >= TBM && g.N >= TBN && g.m_real % 8 == 0 && g.N % 8 == 0) {
      TnPlan pl;
      pl.ntm = (int)((g.m_real + TBM - 1) / TBM);
      pl.ntn = (int)((g.N + TBN - 1) / TBN);
      pl.nsplit = (int)z;
      const int ntile = pl.ntm * pl.ntn;
      const int64_t rounds = (z + 7) / 8;  // slabs per XCD
      if (g.M > g.m_real)
        hipLaunchKernelGGL(gemm_bf16_tn_big_kernel<true>, dim3((unsigned)(8 * rounds * ntile)), dim3(512), 0, s, g, pl);
      else
        hipLaunchKernelGGL(gemm_bf16_tn_big_kernel<false>, dim3((unsigned)(8 * rounds * ntile)), dim3(512), 0, s, g, pl);
      return hip_check(hipGetLastError(), "mrl_gemm_bf16_tn");
    }
  }
  const unsigned gm = (unsigned)((g.M + QBM - 1) / QBM);
  if (g.N <= 32) hipLaunchKernelGGL((gemm_bf16_tn_kernel<32>), dim3(1, gm, (unsigned)z), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_bf16_tn_kernel<128>), dim3((unsigned)((g.N + 127) / 128), gm, (unsigned)z), dim3(256), 0,
                          s, g);
  return hip_check(hipGetLastError(), "mrl_gemm_bf16_tn");
}

int mrl_cast_rows_bf16(const float* x, int64_t rows, int64_t cols, int64_t ldx, uint16_t* y, int64_t ldy,
                       void* stream) {
  if (!x || !y) return fail(E_ARG, "mrl_cast_rows_bf16: null pointer");
  if (ldy < cols) return fail(E_ARG, "mrl_cast_rows_bf16: ldy < cols");
  if (rows <= 0 || ldy <= 0) return OK;
  int64_t gsz = (rows * ldy + 255) / 256;
  if (gsz > 8192) gsz = 8192;
  hipLaunchKernelGGL(cast_rows_bf16_kernel, dim3((unsigned)gsz), dim3(256), 0, (hipStream_t)stream, x, rows, cols, ldx,
                     y, ldy);
  return hip_check(hipGetLastError(), "mrl_cast_rows_bf16");
}

int mrl_pack_w_bf16(const float* w, int64_t din, int64_t dout, int32_t transpose, uint16_t* out, int64_t ld,
                    void* stream) {
  if (!w || !out) return fail(E_ARG, "mrl_pack_w_bf16: null pointer");
  if (ld < (transpose ? din : dout)) return fail(E_ARG, "mrl_pack_w_bf16: ld too small");
  const int64_t total = (transpose ? dout : din) * ld;
  if (total <= 0) return OK;
  int64_t gsz = (total + 255) / 256;
  if (gsz > 4096) gsz = 4096;
  hipLaunchKernelGGL(pack_w_bf16_kernel, dim3((unsigned)gsz), dim3(256), 0, (hipStream_t)stream, w, din, dout, transpose,
                     out, ld);
  return hip_check(hipGetLastError(), "mrl_pack_w_bf16");
}

}  // extern "C"
