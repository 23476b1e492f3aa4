// Advantage scan, standardisation and the device-resident CG / step-scaling /
// line-search vector kernels of the TRPO update.
//
// GAE (core.py:63-75 + misc_utils.py:9-27 `discount` via scipy lfilter): on
// time-major [T, E] rows the per-path reverse recurrences
//     adv_t = delta_t + gamma*lam*cont_t*adv_{t+1},  ret_t = r_t + gamma*cont_t*ret_{t+1}
// are linear, so each (chunk of L steps, env) is summarised as an affine map
// (A, B): adv_in = A + B*adv_out, and chunks compose by a parallel scan.
// One pass: r / v / flags are read once, adv / ret written once (17 B per row).
// Scans run in fp64 like lfilter; outputs are fp32.
#include <math.h>
#include <stdlib.h>

#include "../../include/mrl_hip.h"
#include "mrl_common.h"
#include "fvp_split_role.h"

namespace mrl {

// One block owns GAE_EB envs over the whole horizon: thread (c, e) holds chunk c
// (GAE_L consecutive steps) of env e in registers, so every load of the scan is
// issued up front (a wave instruction covers 4 rows x 64 B) and r / v / flags are
// read from HBM exactly once.  Each chunk is summarised as the affine map of its
// recurrence, one wave per env composes the GAE_NC chunk maps with a reverse
// shuffle scan, and each thread re-runs its chunk from the carried-in value and
// writes adv / ret.  Horizons longer than GAE_NC * L run as segments from the
// last to the first, the carry held by the env's scan wave.
#ifndef MRL_GAE_EB
#define MRL_GAE_EB 16
#endif
#ifndef MRL_GAE_LMAX
#define MRL_GAE_LMAX 32
#endif
#ifndef MRL_GAE_NC
#define MRL_GAE_NC 32
#endif
constexpr int GAE_EB = MRL_GAE_EB;       // envs per block: one 64 B row segment
constexpr int GAE_NC = MRL_GAE_NC;       // chunks per segment: one per lane of a half-wave (32) or wave (64)
static_assert(GAE_NC == 32 || GAE_NC == 64, "scan groups are half-waves or waves");
constexpr int GAE_THREADS = GAE_EB * GAE_NC;
constexpr int GAE_LMAX = MRL_GAE_LMAX;
constexpr int GAE_PITCH = GAE_EB + 1;    // LDS row pitch (doubles): 2-way conflicts at most

template <int L>
__global__ __launch_bounds__(GAE_THREADS) void gae_scan_kernel(const float* __restrict__ rew,
                                                               const float* __restrict__ v,
                                                               const uint8_t* __restrict__ flags, int64_t T,
                                                               int64_t E, double gamma, double lam,
                                                               float* __restrict__ adv, float* __restrict__ ret,
                                                               double* __restrict__ part) {
  __shared__ double sA[GAE_NC * GAE_PITCH], sB[GAE_NC * GAE_PITCH], sR[GAE_NC * GAE_PITCH],
      sC[GAE_NC * GAE_PITCH];
  __shared__ double red[2][GAE_THREADS / 64];
  const int tid = threadIdx.x;
  const int el = tid % GAE_EB, c = tid / GAE_EB;
  const int64_t blk = xcd_segment(blockIdx.x, gridDim.x);  // env segment of this block
  const int64_t e = blk * GAE_EB + el;
  const bool live = e < E;
  const double gl = gamma * lam;
  const int64_t S = (int64_t)GAE_NC * L;
  const int64_t nseg = (T + S - 1) / S;
  const int lane = tid & 63, wave = tid >> 6;
  const int sc = tid % GAE_NC, se = tid / GAE_NC;  // scan: a group of GAE_NC lanes = env slot se, lane = chunk sc
  double carry_a = 0.0, carry_r = 0.0;                    // held by the half-wave of env slot se
  double s1 = 0.0, s2 = 0.0;
  for (int64_t seg = nseg - 1; seg >= 0; --seg) {
    const int64_t t0 = seg * S + (int64_t)c * L;
    // uniform segment/block base + 32-bit per-lane offsets (S * E < 2^29, checked on the host)
    const int64_t base = seg * S * E + blk * GAE_EB;
    const float* rb = rew + base;
    const float* vb = v + base;
    const uint8_t* fb = flags + base;
    // branch-free loads: rows past T and envs past E read a clamped valid element
    // and are masked where they are used
    const int64_t rows = min(S, T - seg * S);  // rows of this segment
    const int elc = (int)min((int64_t)el, E - 1 - blk * GAE_EB);
    auto off = [&](int row) -> uint32_t {  // byte offset of (row, env) from the base, float elements
      const int rc = row < rows ? row : (int)rows - 1;
      return ((uint32_t)rc * (uint32_t)E + (uint32_t)elc) * 4u;
    };
    float rr[L], vv[L];
    uint8_t ff[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint32_t o = off(c * L + j);
      rr[j] = *(const float*)((const char*)rb + o);
      vv[j] = *(const float*)((const char*)vb + o);
      ff[j] = fb[o >> 2];
    }
    const int64_t tn = t0 + L;  // first row of the next chunk (may sit in the next segment)
    const float vnext = (live && tn < T) ? v[tn * E + e] : 0.f;
    // delta_t and the continuation flag of step j of this chunk
    auto step = [&](int j, bool& cont) -> double {
      const int64_t t = t0 + j;
      cont = !(ff[j] & 1) && (t + 1 < T);
      const double vt = (double)vv[j];
      const double vn = (j + 1 < L) ? (double)vv[j + 1 < L ? j + 1 : j] : (double)vnext;
      // bootstrap b1[t+1]: next baseline inside the episode, 0 if terminated, else b[-1] (core.py:73)
      const double boot = cont ? vn : ((ff[j] & 2) ? 0.0 : vt);
      return (double)rr[j] + gamma * boot - vt;
    };
    // chunk summary: adv_in = A + B * adv_out, ret_in = R + C * ret_out
    double A = 0.0, B = 1.0, R = 0.0, Cc = 1.0;
#pragma unroll
    for (int j = L - 1; j >= 0; --j) {
      if (t0 + j < T) {
        bool cont;
        const double d = step(j, cont);
        const double kk = cont ? 1.0 : 0.0;
        A = d + gl * kk * A;
        B = gl * kk * B;
        R = (double)rr[j] + gamma * kk * R;
        Cc = gamma * kk * Cc;
      }
    }
    sA[c * GAE_PITCH + el] = A;
    sB[c * GAE_PITCH + el] = B;
    sR[c * GAE_PITCH + el] = R;
    sC[c * GAE_PITCH + el] = Cc;
    __syncthreads();
    {
      // reverse inclusive scan of the maps of env slot se over its chunks (lane = chunk)
      double a = sA[sc * GAE_PITCH + se], b = sB[sc * GAE_PITCH + se];
      double r = sR[sc * GAE_PITCH + se], cc = sC[sc * GAE_PITCH + se];
#pragma unroll
      for (int off = 1; off < GAE_NC; off <<= 1) {
        const double a2 = __shfl_down(a, off), b2 = __shfl_down(b, off);
        const double r2 = __shfl_down(r, off), c2 = __shfl_down(cc, off);
        if (sc + off < GAE_NC) {
          a = a + b * a2;
          b = b * b2;
          r = r + cc * r2;
          cc = cc * c2;
        }
      }
      // exclusive: the composite of the later chunks, applied to the segment carry
      double xa = __shfl_down(a, 1), xb = __shfl_down(b, 1), xr = __shfl_down(r, 1), xc = __shfl_down(cc, 1);
      if (sc == GAE_NC - 1) { xa = 0.0; xb = 1.0; xr = 0.0; xc = 1.0; }
      const double in_a = xa + xb * carry_a, in_r = xr + xc * carry_r;
      const int l0 = lane & (64 - GAE_NC);  // the group's chunk 0 (lane 32 or 0 of a half-wave, 0 of a wave)
      const double a0 = __shfl(a, l0), b0 = __shfl(b, l0), r0 = __shfl(r, l0), c0 = __shfl(cc, l0);
      carry_a = a0 + b0 * carry_a;
      carry_r = r0 + c0 * carry_r;
      __syncthreads();  // every summary read before the carries overwrite them
      sA[sc * GAE_PITCH + se] = in_a;
      sR[sc * GAE_PITCH + se] = in_r;
    }
    __syncthreads();
    double a = sA[c * GAE_PITCH + el], r = sR[c * GAE_PITCH + el];
    float* ab = adv + base;
    float* tb = ret + base;
#pragma unroll
    for (int j = L - 1; j >= 0; --j) {
      if (live && t0 + j < T) {
        bool cont;
        const double dj = step(j, cont);
        const double kk = cont ? 1.0 : 0.0;
        a = dj + gl * kk * a;
        r = (double)rr[j] + gamma * kk * r;
        const float af = (float)a;
        const uint32_t o = off(c * L + j);
        *(float*)((char*)ab + o) = af;
        *(float*)((char*)tb + o) = (float)r;
        s1 += (double)af;
        s2 += (double)af * (double)af;
      }
    }
    __syncthreads();  // LDS reused by the next (earlier) segment
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off);
    s2 += __shfl_down(s2, off);
  }
  if (lane == 0) {
    red[0][wave] = s1;
    red[1][wave] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int w = 0; w < GAE_THREADS / 64; ++w) {
      t1 += red[0][w];
      t2 += red[1][w];
    }
    part[blk * 2 + 0] = t1;
    part[blk * 2 + 1] = t2;
  }
}

// The exact-fit form (round 6): T = GAE_NC * L (one segment) and E a multiple of GAE_EB
// -- the benchmark's 1024 x 4096.  Same per-row arithmetic and summation order as
// gae_scan_kernel, rebuilt for instruction count (that kernel issues ~100 instructions per
// row: per-lane bounds clamps, 64-bit address arithmetic per load, the delta recomputed
// in the second pass; at 16 K rows per CU its VALU time alone is ~10 us):
//  * no bounds: every load / store is a uniform row base (SGPR) + one per-lane 32-bit
//    offset fixed for the thread's chunk;
//  * loads issued in consumption order (the chunk's last step first), so the summary pass
//    starts on the first rows to land instead of the last;
//  * delta_t kept in registers (fp64) for the second pass; the chunk maps' multipliers
//    B, C are gl^L / gamma^L unless the chunk breaks (0): no per-row products;
//  * the moments' final sum rides in the last block to finish (a ticket counter; the
//    partials handed over as sc1 granules, MI355X_MICROARCH.md's hand-off table, row 1),
//    so there is no second launch.
typedef uint32_t gran4_t __attribute__((ext_vector_type(4)));  // one 16-B granule

template <int L>
__global__ __launch_bounds__(GAE_THREADS) void gae_full_kernel(const float* __restrict__ rew,
                                                               const float* __restrict__ v,
                                                               const uint8_t* __restrict__ flags, int64_t E,
                                                               double gamma, double lam, float* __restrict__ adv,
                                                               float* __restrict__ ret, double* __restrict__ part,
                                                               uint32_t* __restrict__ ticket,
                                                               double* __restrict__ moments, double count) {
  __shared__ double sA[GAE_NC * GAE_PITCH], sB[GAE_NC * GAE_PITCH], sR[GAE_NC * GAE_PITCH],
      sC[GAE_NC * GAE_PITCH];
  __shared__ double red[2][GAE_THREADS];
  __shared__ int is_last;
  const int tid = threadIdx.x;
  const int el = tid % GAE_EB, c = tid / GAE_EB;
  const int64_t blk = xcd_segment(blockIdx.x, gridDim.x);
  const double gl = gamma * lam;
  const int lane = tid & 63, wave = tid >> 6;
  const int sc = tid % GAE_NC, se = tid / GAE_NC;
  // byte offset of (row c*L, env) -- the same for every step j of the chunk; step j adds
  // the uniform j * E * 4 to the base pointer (T * E * 4 < 2^31, checked on the host)
  const uint32_t E4 = (uint32_t)E * 4u;
  const uint32_t o4 = ((uint32_t)(c * L) * (uint32_t)E + (uint32_t)(blk * GAE_EB + el)) * 4u;
  const bool lastc = c == GAE_NC - 1;
  // buffer resources: per access one VGPR offset (o4) + the row's uniform SGPR offset
  const int nbytes = (int)(GAE_NC * L * E4);
  const __amdgpu_buffer_rsrc_t rr_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rew), 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t vv_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(v), 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ff_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(flags), 0, nbytes / 4, 0x00020000);
  float rr[L], vv[L];
  uint32_t ff[L];
#pragma unroll
  for (int j = L - 1; j >= 0; --j) {
    const uint32_t rowb = (uint32_t)j * E4;
    rr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr_rs, o4, rowb, 0));
    vv[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vv_rs, o4, rowb, 0));
    ff[j] = __builtin_amdgcn_raw_buffer_load_b8(ff_rs, o4 >> 2, rowb >> 2, 0);
  }
  // v of the next chunk's first row (the last chunk's is never used: t + 1 = T)
  const float vnext = __builtin_bit_cast(
      float, __builtin_amdgcn_raw_buffer_load_b32(vv_rs, lastc ? o4 : o4 + (uint32_t)L * E4, 0, 0));
  double glL = 1.0, gL = 1.0;  // B, C of an unbroken chunk: the products gae_scan_kernel forms
#pragma unroll
  for (int j = 0; j < L; ++j) {
    glL = gl * glL;
    gL = gamma * gL;
  }
  double dd[L];
  double A = 0.0, R = 0.0;
  bool brk = false;
  double vn = (double)vnext;
  uint32_t fl[(L + 15) / 16] = {};  // the flags again, 2 bits per step, for the second pass
#pragma unroll
  for (int j = L - 1; j >= 0; --j) {
    fl[j >> 4] |= ff[j] << (2 * (j & 15));
    const bool cont = !(ff[j] & 1u) && !(lastc && j == L - 1);
    const double vt = (double)vv[j], rj = (double)rr[j];
    // bootstrap b1[t+1]: next baseline inside the episode, 0 if terminated, else b[-1] (core.py:73)
    const double boot = cont ? vn : ((ff[j] & 2u) ? 0.0 : vt);
    const double d = rj + gamma * boot - vt;
    dd[j] = d;
    A = d + (cont ? gl : 0.0) * A;
    R = rj + (cont ? gamma : 0.0) * R;
    brk = brk || !cont;
    vn = vt;
  }
  sA[c * GAE_PITCH + el] = A;
  sB[c * GAE_PITCH + el] = brk ? 0.0 : glL;
  sR[c * GAE_PITCH + el] = R;
  sC[c * GAE_PITCH + el] = brk ? 0.0 : gL;
  __syncthreads();
  {
    // reverse inclusive scan of env slot se's chunk maps (lane = chunk), as gae_scan_kernel
    double a = sA[sc * GAE_PITCH + se], b = sB[sc * GAE_PITCH + se];
    double r = sR[sc * GAE_PITCH + se], cc = sC[sc * GAE_PITCH + se];
#pragma unroll
    for (int off = 1; off < GAE_NC; off <<= 1) {
      const double a2 = __shfl_down(a, off), b2 = __shfl_down(b, off);
      const double r2 = __shfl_down(r, off), c2 = __shfl_down(cc, off);
      if (sc + off < GAE_NC) {
        a = a + b * a2;
        b = b * b2;
        r = r + cc * r2;
        cc = cc * c2;
      }
    }
    double xa = __shfl_down(a, 1), xb = __shfl_down(b, 1), xr = __shfl_down(r, 1), xc = __shfl_down(cc, 1);
    if (sc == GAE_NC - 1) { xa = 0.0; xb = 1.0; xr = 0.0; xc = 1.0; }
    const double in_a = xa + xb * 0.0, in_r = xr + xc * 0.0;
    __syncthreads();
    sA[sc * GAE_PITCH + se] = in_a;
    sR[sc * GAE_PITCH + se] = in_r;
  }
  __syncthreads();
  double a = sA[c * GAE_PITCH + el], r = sR[c * GAE_PITCH + el];
  double s1 = 0.0, s2 = 0.0;
  const __amdgpu_buffer_rsrc_t adv_rs = __builtin_amdgcn_make_buffer_rsrc(adv, 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ret_rs = __builtin_amdgcn_make_buffer_rsrc(ret, 0, nbytes, 0x00020000);
#pragma unroll
  for (int j = L - 1; j >= 0; --j) {
    const bool cont = !((fl[j >> 4] >> (2 * (j & 15))) & 1u) && !(lastc && j == L - 1);
    a = dd[j] + (cont ? gl : 0.0) * a;
    r = (double)rr[j] + (cont ? gamma : 0.0) * r;
    const float af = (float)a;
    const uint32_t rowb = (uint32_t)j * E4;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, af), adv_rs, o4, rowb, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, (float)r), ret_rs, o4, rowb, 0);
    s1 += (double)af;
    s2 += (double)af * (double)af;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off);
    s2 += __shfl_down(s2, off);
  }
  if (lane == 0) {
    red[0][wave] = s1;
    red[1][wave] = s2;
  }
  __syncthreads();
  const int64_t nb = gridDim.x;
  __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(part, 0, (int)(nb * 16), 0x00020000);
  if (tid == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int w = 0; w < GAE_THREADS / 64; ++w) {
      t1 += red[0][w];
      t2 += red[1][w];
    }
    // the block's partial as one sc1 granule, waited for, then the ticket (agent scope)
    const uint64_t b1 = (uint64_t)__double_as_longlong(t1), b2 = (uint64_t)__double_as_longlong(t2);
    const gran4_t g = {(uint32_t)b1, (uint32_t)(b1 >> 32), (uint32_t)b2, (uint32_t)(b2 >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(g, prs, (uint32_t)(blk * 16), 0, 16);  // aux 16 = sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t done = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = done == (uint32_t)(nb - 1);
  }
  __syncthreads();
  if (!is_last) return;
  // the last block: every partial through sc1 loads, summed in block order in a fixed
  // tree (the order moments_final_kernel uses, over GAE_THREADS lanes)
  double t1 = 0.0, t2 = 0.0;
  for (int64_t i = tid; i < nb; i += GAE_THREADS) {
    const gran4_t g = __builtin_amdgcn_raw_buffer_load_b128(prs, (uint32_t)(i * 16), 0, 16);
    t1 += __longlong_as_double((long long)(((uint64_t)g.y << 32) | g.x));
    t2 += __longlong_as_double((long long)(((uint64_t)g.w << 32) | g.z));
  }
  red[0][tid] = t1;
  red[1][tid] = t2;
  __syncthreads();
  for (int o = GAE_THREADS / 2; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    moments[0] = red[0][0];
    moments[1] = red[1][0];
    moments[2] = count;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
  }
}

__global__ void moments_final_kernel(const double* __restrict__ part, int64_t nb, double count,
                                     double* __restrict__ moments) {
  __shared__ double red[2][256];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = threadIdx.x; i < nb; i += 256) {
    s1 += part[i * 2];
    s2 += part[i * 2 + 1];
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    moments[0] = red[0][0];
    moments[1] = red[1][0];
    moments[2] = count;
  }
}

// mom = (sum, sumsq, n) of the first pass; cmom = (sum, sumsq, n) of (adv - mom[0]/mom[2]),
// the second pass of numpy's two-pass std (core.py:100-105): the centred sums do not
// cancel when |mean| >> std.  Without cmom the single-pass form is used.
__global__ void standardize_kernel(float* __restrict__ adv, int64_t n, const double* __restrict__ mom,
                                   const double* __restrict__ cmom) {
  const double mean0 = mom[0] / mom[2];
  double mean, var;
  if (cmom) {
    const double d = cmom[0] / cmom[2];  // residual of the shift (rounding of mean0)
    mean = mean0 + d;
    var = fmax(cmom[1] / cmom[2] - d * d, 0.0);
  } else {
    mean = mean0;
    var = fmax(mom[1] / mom[2] - mean * mean, 0.0);
  }
  const double stdv = sqrt(var);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adv[i] = (float)(((double)adv[i] - mean) / stdv);
}

__global__ void vf_target_kernel(const float* __restrict__ ret, const float* __restrict__ vp, double mixfrac, int64_t n,
                                 float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (float)((double)ret[i] * mixfrac + (double)vp[i] * (1.0 - mixfrac));
}

// ------------------------------------------------------------------ CG (one workgroup)
constexpr int CG_T = 1024;
#ifndef MRL_CG_REG  // 1: the single-block CG update keeps its slices in registers (n <= 8192)
#define MRL_CG_REG 1
#endif

// The sum of the block's CG_T values as the pairwise tree red[i] += red[i + o],
// o = CG_T/2 .. 1, adds them (the tree every CG kernel's results are defined by), in
// two barriers instead of eleven: wave 0 lane i gathers its 16 values v[i + 64 k] and
// adds them in the tree's cross-wave order (o = 512 .. 64: k with k + 8, k + 4, k + 2,
// k + 1), then o = 32 .. 1 as lane shuffles.  red: CG_T + 1 doubles (the result slot
// red[CG_T] is only written after the first barrier, so back-to-back sums need no third).
__device__ inline double block_sum(double v, double* red) {
  static_assert(CG_T == 1024, "the cross-wave tree below is CG_T = 16 x 64");
  red[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    const double* q = red + threadIdx.x;
    // b[k] = (v[k] + v[k + 8]) + (v[k + 4] + v[k + 12]) (in units of 64), one k at a time
    auto quad = [&](int k) { return (q[64 * k] + q[64 * (k + 8)]) + (q[64 * (k + 4)] + q[64 * (k + 12)]); };
    // (the fences keep the gathers one quad at a time: four doubles in flight, not
    // sixteen, beside the CG kernels' register-resident vectors)
    const double b0 = quad(0);
    asm volatile("" ::: "memory");
    const double c0 = b0 + quad(2);
    asm volatile("" ::: "memory");
    const double b1 = quad(1);
    asm volatile("" ::: "memory");
    double t = c0 + (b1 + quad(3));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    if (threadIdx.x == 0) red[CG_T] = t;
  }
  __syncthreads();
  return red[CG_T];
}

__global__ __launch_bounds__(CG_T) void cg_init_kernel(const double* __restrict__ b, int64_t n, double* x, double* r,
                                                       double* p, float* p32, double* ax, double* state,
                                                       int32_t* flag) {
  __shared__ double red[CG_T + 1];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    const double bi = b[i];
    x[i] = 0.0;
    if (ax) ax[i] = 0.0;
    r[i] = bi;
    p[i] = bi;
    p32[i] = (float)bi;
    s += bi * bi;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    state[0] = s;
    state[1] = 0.0;
    state[2] = 0.0;
    flag[0] = 0;
    flag[1] = 0;
  }
}

__global__ __launch_bounds__(CG_T) void cg_update_kernel(const float* __restrict__ fvp, double damping, double tol,
                                                         int64_t n, double* x, double* r, double* p, float* p32,
                                                         double* ax, double* state, int32_t* flag) {
  __shared__ double red[CG_T + 1];
  if (flag[0] != 0) return;
  const double rdotr = state[0];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    const double z = (double)fvp[i] + damping * p[i];
    s += p[i] * z;
  }
  const double pz = block_sum(s, red);
  const double v = rdotr / pz;
  s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    const double pi = p[i];
    const double z = (double)fvp[i] + damping * pi;
    x[i] += v * pi;
    if (ax) ax[i] += v * z;  // A x = sum_k v_k A p_k: the step scaling needs no extra Fisher product
    const double ri = r[i] - v * z;
    r[i] = ri;
    s += ri * ri;
  }
  const double newr = block_sum(s, red);
  const double mu = newr / rdotr;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    const double pi = r[i] + mu * p[i];
    p[i] = pi;
    p32[i] = (float)pi;
  }
  if (threadIdx.x == 0) {
    state[0] = newr;
    state[1] = pz;
    state[2] += 1.0;
    if (newr < tol) flag[0] = 1;
  }
}

// The same update with each thread's K-element slice of p / r / x / A x held in
// registers: every operand is loaded once, up front, instead of once per pass
// (three dependent global passes of the plain kernel).  Per-thread accumulation
// order and the block_sum tree are the plain kernel's, so the results are identical.
// PACK: the next Fisher product's tangent image too -- the split image of p32
// (split_image_item, as mlp_pack_split_kernel writes it), one launch instead of two
struct CgPack {
  MlpDims d;
  BDims b;
  float* image;
};

template <int K, bool PACK>
__device__ inline void cg_update_reg_body(const float* fvp, double damping, double tol, int64_t n, double* x,
                                          double* r, double* p, float* p32, double* ax, double* state, int32_t* flag,
                                          const CgPack& pk, double* red) {
  const double rdotr = state[0];
  // z = fvp + damping p is recomputed where it is used (the same value) from the f32 fvp
  // kept in registers: 8 VGPRs fewer than a double z, no spills at CG_T threads
  double pr[K], rr[K], xr[K], ar[K];
  float fr[K];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t i = threadIdx.x + (int64_t)k * CG_T;
    pr[k] = rr[k] = xr[k] = ar[k] = 0.0;
    fr[k] = 0.f;
    if (i < n) {
      const double pi = p[i];
      fr[k] = fvp[i];
      const double z = (double)fr[k] + damping * pi;
      pr[k] = pi;
      rr[k] = r[i];
      xr[k] = x[i];
      if (ax) ar[k] = ax[i];
      s += pi * z;
    }
  }
  const double pz = block_sum(s, red);
  const double v = rdotr / pz;
  s = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t i = threadIdx.x + (int64_t)k * CG_T;
    if (i < n) {
      const double z = (double)fr[k] + damping * pr[k];
      x[i] = xr[k] + v * pr[k];
      if (ax) ax[i] = ar[k] + v * z;
      const double ri = rr[k] - v * z;
      r[i] = ri;
      rr[k] = ri;
      s += ri * ri;
    }
  }
  const double newr = block_sum(s, red);
  const double mu = newr / rdotr;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t i = threadIdx.x + (int64_t)k * CG_T;
    if (i < n) {
      const double pi = rr[k] + mu * pr[k];
      p[i] = pi;
      p32[i] = (float)pi;
    }
  }
  if (threadIdx.x == 0) {
    state[0] = newr;
    state[1] = pz;
    state[2] += 1.0;
    if (newr < tol) flag[0] = 1;
  }
  if constexpr (PACK) {
    // the new p32 staged in LDS (8192 floats), read there by the image gathers
    __shared__ float sp[8 * CG_T];
#pragma unroll
    for (int k = 0; k < K; ++k) sp[threadIdx.x + k * CG_T] = (float)(rr[k] + mu * pr[k]);
    __syncthreads();
    const int items = split_image_items(pk.b);
    for (int u = threadIdx.x; u < items; u += CG_T) split_image_item(pk.d, pk.b, sp, pk.image, u);
  }
}

template <int K, bool PACK = false>
__global__ __launch_bounds__(CG_T) void cg_update_reg_kernel(const float* __restrict__ fvp, double damping, double tol,
                                                             int64_t n, double* x, double* r, double* p, float* p32,
                                                             double* ax, double* state, int32_t* flag,
                                                             CgPack pk = CgPack{}) {
  __shared__ double red[CG_T + 1];
  if (flag[0] != 0) return;
  cg_update_reg_body<K, PACK>(fvp, damping, tol, n, x, r, p, p32, ax, state, flag, pk, red);
}


__global__ __launch_bounds__(CG_T) void trpo_step_kernel(const float* __restrict__ fvp, const double* __restrict__ x,
                                                         const float* __restrict__ g, double damping, double max_kl,
                                                         int64_t n, double* fullstep, double* out) {
  __shared__ double red[CG_T + 1];
  double s = 0.0, sg = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    s += x[i] * ((double)fvp[i] + damping * x[i]);
    sg += (double)g[i] * x[i];
  }
  const double xFx = block_sum(s, red);
  const double gx = block_sum(sg, red);
  const double shs = 0.5 * xFx;
  const double lm = sqrt(shs / max_kl);
  for (int64_t i = threadIdx.x; i < n; i += CG_T) fullstep[i] = x[i] / lm;
  if (threadIdx.x == 0) {
    out[0] = shs;
    out[1] = lm;
    out[2] = -gx;
    out[3] = -gx / lm;
  }
}

// same scaling from A x accumulated by the CG updates (A linear: A sum v_k p_k = sum v_k z_k)
__global__ __launch_bounds__(CG_T) void trpo_step_ax_kernel(const double* __restrict__ ax, const double* __restrict__ x,
                                                            const float* __restrict__ g, double max_kl, int64_t n,
                                                            double* fullstep, double* out) {
  __shared__ double red[CG_T + 1];
  double s = 0.0, sg = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    s += x[i] * ax[i];
    sg += (double)g[i] * x[i];
  }
  const double xAx = block_sum(s, red);
  const double gx = block_sum(sg, red);
  const double shs = 0.5 * xAx;
  const double lm = sqrt(shs / max_kl);
  for (int64_t i = threadIdx.x; i < n; i += CG_T) fullstep[i] = x[i] / lm;
  if (threadIdx.x == 0) {
    out[0] = shs;
    out[1] = lm;
    out[2] = -gx;
    out[3] = -gx / lm;
  }
}

// ---- multi-block CG / step scaling for large n (wide nets: Humanoid P = 727,074).
// The single-block kernels above stream n fp64 elements through one CU (1.6 ms per
// CG update at P = 727 k); here each of CGB blocks owns one contiguous chunk, block
// partial sums go to a scratch area of `state` / `out` (mrl_cg_state_doubles), and
// every block reduces the CGB partials in the same fixed order, so all blocks derive
// bit-identical scalars.  The scalars and the flag are written by a 1-thread kernel
// after the last pass, so no block ever reads a value this update is writing.
constexpr int CGB = 256;                    // blocks of the multi-block passes
constexpr int CGB_T = 256;                  // threads per block
constexpr int64_t CG_SMALL_N = 65536;       // n at or below: the single-block kernels
constexpr int CG_SCALARS = 8;               // state[0..7]; partials from state[8]

__device__ inline void cg_chunk(int64_t n, int64_t& lo, int64_t& hi) {
  const int64_t chunk = ((n + CGB - 1) / CGB + CGB_T - 1) / CGB_T * CGB_T;
  lo = (int64_t)blockIdx.x * chunk;
  hi = min(n, lo + chunk);
}
__device__ inline double blk_sum(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = CGB_T / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
// sum of the CGB partials part[0..CGB) in a fixed order (identical in every block)
__device__ inline double part_sum(const double* part, double* red) {
  return blk_sum(threadIdx.x < CGB ? part[threadIdx.x] : 0.0, red);
}

__global__ __launch_bounds__(CGB_T) void cgm_init_kernel(const double* __restrict__ b, int64_t n, double* x, double* r,
                                                          double* p, float* p32, double* ax, double* part) {
  __shared__ double red[CGB_T];
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  double s = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) {
    const double bi = b[i];
    x[i] = 0.0;
    if (ax) ax[i] = 0.0;
    r[i] = bi;
    p[i] = bi;
    p32[i] = (float)bi;
    s += bi * bi;
  }
  s = blk_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ __launch_bounds__(CGB_T) void cgm_init_final_kernel(double* state, int32_t* flag) {
  __shared__ double red[CGB_T];
  const double s = part_sum(state + CG_SCALARS, red);
  if (threadIdx.x == 0) {
    state[0] = s;
    state[1] = 0.0;
    state[2] = 0.0;
    flag[0] = 0;
    flag[1] = 0;
  }
}
// pass 1: p.z partials
__global__ __launch_bounds__(CGB_T) void cgm_pz_kernel(const float* __restrict__ fvp, double damping, int64_t n,
                                                        const double* __restrict__ p, double* state,
                                                        const int32_t* flag) {
  __shared__ double red[CGB_T];
  if (flag[0] != 0) return;
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  double s = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) s += p[i] * ((double)fvp[i] + damping * p[i]);
  s = blk_sum(s, red);
  if (threadIdx.x == 0) state[CG_SCALARS + blockIdx.x] = s;
}
// pass 2: v = rdotr / p.z; x += v p; ax += v z; r -= v z; r.r partials
__global__ __launch_bounds__(CGB_T) void cgm_xr_kernel(const float* __restrict__ fvp, double damping, int64_t n,
                                                        double* x, double* r, const double* __restrict__ p,
                                                        double* ax, double* state, const int32_t* flag) {
  __shared__ double red[CGB_T];
  if (flag[0] != 0) return;
  const double v = state[0] / part_sum(state + CG_SCALARS, red);
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  double s = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) {
    const double pi = p[i];
    const double z = (double)fvp[i] + damping * pi;
    x[i] += v * pi;
    if (ax) ax[i] += v * z;
    const double ri = r[i] - v * z;
    r[i] = ri;
    s += ri * ri;
  }
  s = blk_sum(s, red);
  if (threadIdx.x == 0) state[CG_SCALARS + CGB + blockIdx.x] = s;
}
// pass 3: mu = r.r / rdotr; p = r + mu p
__global__ __launch_bounds__(CGB_T) void cgm_p_kernel(int64_t n, const double* __restrict__ r, double* p, float* p32,
                                                       const double* state, const int32_t* flag) {
  __shared__ double red[CGB_T];
  if (flag[0] != 0) return;
  const double mu = part_sum(state + CG_SCALARS + CGB, red) / state[0];
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) {
    const double pi = r[i] + mu * p[i];
    p[i] = pi;
    p32[i] = (float)pi;
  }
}
__global__ __launch_bounds__(CGB_T) void cgm_final_kernel(double tol, double* state, int32_t* flag) {
  __shared__ double red[CGB_T];
  if (flag[0] != 0) return;
  const double pz = part_sum(state + CG_SCALARS, red);
  const double newr = part_sum(state + CG_SCALARS + CGB, red);
  if (threadIdx.x == 0) {
    state[0] = newr;
    state[1] = pz;
    state[2] += 1.0;
    if (newr < tol) flag[0] = 1;
  }
}
// step scaling: x.ax and g.x partials, then every block derives shs / lm and writes its
// chunk of fullstep = x / lm (block 0 the scalars)
__global__ __launch_bounds__(CGB_T) void cgm_step_part_kernel(const double* __restrict__ ax,
                                                               const double* __restrict__ x, const float* __restrict__ g,
                                                               int64_t n, double* out) {
  __shared__ double red[CGB_T];
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  double s = 0.0, sg = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) {
    s += x[i] * ax[i];
    sg += (double)g[i] * x[i];
  }
  s = blk_sum(s, red);
  sg = blk_sum(sg, red);
  if (threadIdx.x == 0) {
    out[CG_SCALARS + blockIdx.x] = s;
    out[CG_SCALARS + CGB + blockIdx.x] = sg;
  }
}
__global__ __launch_bounds__(CGB_T) void cgm_step_kernel(const double* __restrict__ x, double max_kl, int64_t n,
                                                          double* fullstep, double* out) {
  __shared__ double red[CGB_T];
  const double xAx = part_sum(out + CG_SCALARS, red);
  const double gx = part_sum(out + CG_SCALARS + CGB, red);
  const double shs = 0.5 * xAx;
  const double lm = sqrt(shs / max_kl);
  int64_t lo, hi;
  cg_chunk(n, lo, hi);
  for (int64_t i = lo + threadIdx.x; i < hi; i += CGB_T) fullstep[i] = x[i] / lm;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = shs;
    out[1] = lm;
    out[2] = -gx;
    out[3] = -gx / lm;
  }
}

__global__ void axpy_cast_kernel(const float* __restrict__ a, const double* __restrict__ b, double frac, int64_t n,
                                 float* __restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = (float)((double)a[i] + frac * b[i]);
}

// K line-search candidates (trpo.py:149-150): row k = (float)(theta_old + 0.5^(k0+k) fullstep)
// -- axpy_cast_kernel's arithmetic per row (linesearch's stepfrac is an exact power of two)
__global__ void ls_candidates_kernel(const float* __restrict__ a, const double* __restrict__ b, int k0, int K,
                                     int64_t n, float* __restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double ai = (double)a[i], bi = b[i];
    for (int k = 0; k < K; ++k) o[(int64_t)k * n + i] = (float)(ai + ldexp(1.0, -(k0 + k)) * bi);
  }
}

// Adam step in floatX (ppo.py:231-258): m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// theta -= a_t m / (sqrt(v) + eps), a_t = lr sqrt(1-b2^t)/(1-b1^t) from the host
__global__ void adam_kernel(float* __restrict__ th, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, float a_t, float b1, float b2, float eps, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * (gi * gi);
    m[i] = mi;
    v[i] = vi;
    th[i] = th[i] - a_t * mi / (sqrtf(vi) + eps);
  }
}

// dst row i = src row idx[i] (rows of `words` 32-bit words): minibatch gathers
__global__ void gather_rows_kernel(const uint32_t* __restrict__ src, const int64_t* __restrict__ idx, int64_t n,
                                   int64_t words, uint32_t* __restrict__ dst) {
  const int64_t total = n * words;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / words, c = i - r * words;
    dst[i] = src[idx[r] * words + c];
  }
}

__global__ void cast_scale_kernel(const float* __restrict__ a, double s, int64_t n, double* __restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = s * (double)a[i];
}

// ------------------------------------------------------------------ moments / episode stats
// per-block fp64 (sum, sumsq) of (a - b - shift) -> part[block][2]; shift = center[0] /
// center[2] (a previous pass's mean) or 0
__global__ void moments_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                               const double* __restrict__ center, double* __restrict__ part) {
  __shared__ double red[2][256];
  const double shift = center ? center[0] / center[2] : 0.0;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = (double)a[i] - (b ? (double)b[i] : 0.0) - shift;
    s1 += v;
    s2 += v * v;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2] = red[0][0];
    part[blockIdx.x * 2 + 1] = red[1][0];
  }
}

// episode statistics over time-major rows (core.py:31-44), blocked like the GAE scan:
// thread (c, e) reads chunk c (L steps) of env e once, counts the episodes that start
// and end inside its chunk and summarises the rest as (head: rows up to its first
// episode end, tail: rows after its last); one walker thread per env then joins the
// chunk summaries in time order, carrying the open episode across chunks and
// segments.  part[block][8] = (n_ep, sum R, sum R^2, max R, sum L, max L, 0, 0)
constexpr int EPS_EB = 16, EPS_NC = 32, EPS_THREADS = EPS_EB * EPS_NC, EPS_PITCH = EPS_EB + 1;

struct EpAcc {
  double cnt = 0, sr = 0, sr2 = 0, mr = -INFINITY, sl = 0, ml = 0;
  __device__ void add(double r, double len) {
    cnt += 1.0;
    sr += r;
    sr2 += r * r;
    mr = fmax(mr, r);
    sl += len;
    ml = fmax(ml, len);
  }
};

template <int L>
__global__ __launch_bounds__(EPS_THREADS) void episode_stats_kernel(const float* __restrict__ rew,
                                                                    const uint8_t* __restrict__ flags, int64_t T,
                                                                    int64_t E, double* __restrict__ part) {
  __shared__ double sHR[EPS_NC * EPS_PITCH], sTR[EPS_NC * EPS_PITCH];
  __shared__ int sHL[EPS_NC * EPS_PITCH], sTL[EPS_NC * EPS_PITCH];
  __shared__ double red[6][EPS_THREADS / 64];
  const int tid = threadIdx.x;
  const int el = tid % EPS_EB, c = tid / EPS_EB;
  const int64_t blk = xcd_segment(blockIdx.x, gridDim.x);  // env segment of this block
  const bool live = blk * EPS_EB + el < E;
  const int64_t S = (int64_t)EPS_NC * L;
  const int64_t nseg = (T + S - 1) / S;
  const int elc = (int)min((int64_t)el, E - 1 - blk * EPS_EB);
  EpAcc acc;
  double open_r = 0.0;  // walker (tid < EPS_EB): the episode still open at the segment start
  int open_len = 0;
  for (int64_t seg = 0; seg < nseg; ++seg) {
    const int64_t base = seg * S * E + blk * EPS_EB;
    const int64_t rows = min(S, T - seg * S);
    float rr[L];
    uint8_t ff[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int row = c * L + j;
      const int rc = row < rows ? row : (int)rows - 1;
      const uint32_t o = (uint32_t)rc * (uint32_t)E + (uint32_t)elc;
      rr[j] = rew[base + o];
      ff[j] = flags[base + o];
    }
    double cur = 0.0, hr = 0.0;
    int clen = 0, hl = 0;
    bool seen = false;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      if (live && c * L + j < rows) {
        cur += (double)rr[j];
        clen += 1;
        if (ff[j] & 1) {
          if (!seen) {
            hr = cur;
            hl = clen;
            seen = true;
          } else {
            acc.add(cur, (double)clen);
          }
          cur = 0.0;
          clen = 0;
        }
      }
    }
    // head = rows through the first end (or the whole chunk: tail length -1 marks "no end")
    sHR[c * EPS_PITCH + el] = seen ? hr : cur;
    sHL[c * EPS_PITCH + el] = seen ? hl : clen;
    sTR[c * EPS_PITCH + el] = cur;
    sTL[c * EPS_PITCH + el] = seen ? clen : -1;
    __syncthreads();
    if (tid < EPS_EB && live) {
      for (int cc = 0; cc < EPS_NC; ++cc) {
        const double h = sHR[cc * EPS_PITCH + tid];
        const int hlen = sHL[cc * EPS_PITCH + tid];
        const int tl = sTL[cc * EPS_PITCH + tid];
        if (tl >= 0) {
          acc.add(open_r + h, (double)(open_len + hlen));
          open_r = sTR[cc * EPS_PITCH + tid];
          open_len = tl;
        } else {
          open_r += h;
          open_len += hlen;
        }
      }
    }
    __syncthreads();
  }
  // block reduction: sums and maxima
  double v[6] = {acc.cnt, acc.sr, acc.sr2, acc.mr, acc.sl, acc.ml};
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const double o = __shfl_down(v[q], off);
      v[q] = (q == 3 || q == 5) ? fmax(v[q], o) : v[q] + o;
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  if (lane == 0)
    for (int q = 0; q < 6; ++q) red[q][wave] = v[q];
  __syncthreads();
  if (tid < 8) {
    double r = 0.0;
    if (tid < 6) {
      r = (tid == 3 || tid == 5) ? -INFINITY : 0.0;
      for (int w = 0; w < EPS_THREADS / 64; ++w) r = (tid == 3 || tid == 5) ? fmax(r, red[tid][w]) : r + red[tid][w];
    }
    part[blk * 8 + tid] = r;
  }
}

__global__ void episode_stats_final_kernel(const double* __restrict__ part, int64_t nb, double* __restrict__ out) {
  // one wave: lane-strided partial sums / maxima over the blocks, then a shuffle tree
  const int lane = threadIdx.x;
  double a[6] = {0, 0, 0, -INFINITY, 0, 0};
  for (int64_t b = lane; b < nb; b += 64) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const double v = part[b * 8 + q];
      a[q] = (q == 3 || q == 5) ? fmax(a[q], v) : a[q] + v;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const double o = __shfl_down(a[q], off);
      a[q] = (q == 3 || q == 5) ? fmax(a[q], o) : a[q] + o;
    }
  }
  if (lane == 0)
    for (int q = 0; q < 6; ++q) out[q] = a[q];
}

static inline int64_t grid_for(int64_t n, int64_t bs = 256, int64_t cap = 2048) {
  int64_t g = (n + bs - 1) / bs;
  if (g < 1) g = 1;
  return g > cap ? cap : g;
}

}  // namespace mrl

using namespace mrl;

extern "C" {

// workspace: [nb fp64 (sum, sumsq) block partials][pad to 64 B][u32 completion ticket]
static int64_t gae_ticket_offset(int64_t E) {
  const int64_t nb = (E + GAE_EB - 1) / GAE_EB;
  return (nb * 2 * (int64_t)sizeof(double) + 63) / 64 * 64;
}

int64_t mrl_gae_workspace_bytes(int64_t T, int64_t E) {
  (void)T;
  if (E <= 0) return 128;
  return gae_ticket_offset(E) + 64;
}

int mrl_gae(const float* rew, const float* vpred, const uint8_t* flags, int64_t T, int64_t E, double gamma, double lam,
            float* adv, float* ret, double* moments, void* workspace, void* stream) {
  if (!rew || !vpred || !flags || !adv || !ret || !moments || !workspace) return fail(E_ARG, "null pointer");
  if (T <= 0 || E <= 0) return OK;
  const int64_t nb = (E + GAE_EB - 1) / GAE_EB;
  if ((int64_t)GAE_NC * GAE_LMAX * (E + GAE_EB) >= ((int64_t)1 << 29))
    return fail(E_UNSUPPORTED, "mrl_gae: E too large for 32-bit segment offsets");
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  // chunk length: the smallest power of two that covers T in one segment, at most GAE_LMAX
  int L = 1;
  while (L < GAE_LMAX && (int64_t)GAE_NC * L < T) L <<= 1;
  // MRL_GAE_GENERAL=1 (tests / A-B probes): the general kernel for every shape
  static const bool general_only = getenv("MRL_GAE_GENERAL") && getenv("MRL_GAE_GENERAL")[0] == '1';
  if (!general_only && T == (int64_t)GAE_NC * L && E % GAE_EB == 0 && T * E * 4 < ((int64_t)1 << 31)) {
    // exact fit: one pass, the moments finished by the last block (gae_full_kernel)
    uint32_t* ticket = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(workspace) + gae_ticket_offset(E));
#define MRL_GAE_FULL(LL)                                                                                          \
  hipLaunchKernelGGL(gae_full_kernel<LL>, dim3(nb), dim3(GAE_THREADS), 0, s, rew, vpred, flags, E, gamma, lam, adv, \
                     ret, part, ticket, moments, (double)(T * E))
    switch (L) {
      case 1: MRL_GAE_FULL(1); break;
      case 2: MRL_GAE_FULL(2); break;
      case 4: MRL_GAE_FULL(4); break;
      case 8: MRL_GAE_FULL(8); break;
      case 16: MRL_GAE_FULL(16); break;
      default: MRL_GAE_FULL(32); break;
    }
#undef MRL_GAE_FULL
    return hip_check(hipGetLastError(), "mrl_gae");
  }
#define MRL_GAE_LAUNCH(LL)                                                                                      \
  hipLaunchKernelGGL(gae_scan_kernel<LL>, dim3(nb), dim3(GAE_THREADS), 0, s, rew, vpred, flags, T, E, gamma, lam, \
                     adv, ret, part)
  switch (L) {
    case 1: MRL_GAE_LAUNCH(1); break;
    case 2: MRL_GAE_LAUNCH(2); break;
    case 4: MRL_GAE_LAUNCH(4); break;
    case 8: MRL_GAE_LAUNCH(8); break;
    case 16: MRL_GAE_LAUNCH(16); break;
    default: MRL_GAE_LAUNCH(32); break;
  }
#undef MRL_GAE_LAUNCH
  hipLaunchKernelGGL(moments_final_kernel, dim3(1), dim3(256), 0, s, part, nb, (double)(T * E), moments);
  return hip_check(hipGetLastError(), "mrl_gae");
}

int mrl_standardize(float* adv, int64_t n, const double* moments, const double* cmoments, void* stream) {
  if (!adv || !moments) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(standardize_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, adv, n, moments,
                     cmoments);
  return hip_check(hipGetLastError(), "mrl_standardize");
}

int mrl_vf_target(const float* ret, const float* vpred, double mixfrac, int64_t n, float* y, void* stream) {
  if (!ret || !vpred || !y) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(vf_target_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ret, vpred, mixfrac, n, y);
  return hip_check(hipGetLastError(), "mrl_vf_target");
}

int64_t mrl_cg_state_doubles(int64_t n) { return n > CG_SMALL_N ? CG_SCALARS + 2 * CGB : 4; }

int mrl_cg_init(const double* b, int64_t n, double* x, double* r, double* p, float* p32, double* ax, double* state,
                int32_t* flag, void* stream) {
  if (!b || !x || !r || !p || !p32 || !state || !flag) return fail(E_ARG, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (n > CG_SMALL_N) {
    hipLaunchKernelGGL(cgm_init_kernel, dim3(CGB), dim3(CGB_T), 0, s, b, n, x, r, p, p32, ax, state + CG_SCALARS);
    hipLaunchKernelGGL(cgm_init_final_kernel, dim3(1), dim3(CGB_T), 0, s, state, flag);
  } else {
    hipLaunchKernelGGL(cg_init_kernel, dim3(1), dim3(CG_T), 0, s, b, n, x, r, p, p32, ax, state, flag);
  }
  return hip_check(hipGetLastError(), "mrl_cg_init");
}

int mrl_cg_update(const float* fvp, double damping, double residual_tol, int64_t n, double* x, double* r, double* p,
                  float* p32, double* ax, double* state, int32_t* flag, void* stream) {
  if (!fvp || !x || !r || !p || !p32 || !state || !flag) return fail(E_ARG, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (n > CG_SMALL_N) {
    hipLaunchKernelGGL(cgm_pz_kernel, dim3(CGB), dim3(CGB_T), 0, s, fvp, damping, n, p, state, flag);
    hipLaunchKernelGGL(cgm_xr_kernel, dim3(CGB), dim3(CGB_T), 0, s, fvp, damping, n, x, r, p, ax, state, flag);
    hipLaunchKernelGGL(cgm_p_kernel, dim3(CGB), dim3(CGB_T), 0, s, n, r, p, p32, state, flag);
    hipLaunchKernelGGL(cgm_final_kernel, dim3(1), dim3(CGB_T), 0, s, residual_tol, state, flag);
  } else if (MRL_CG_REG && n <= 8 * CG_T) {
    hipLaunchKernelGGL(cg_update_reg_kernel<8>, dim3(1), dim3(CG_T), 0, s, fvp, damping, residual_tol, n, x, r, p,
                       p32, ax, state, flag);
  } else {
    hipLaunchKernelGGL(cg_update_kernel, dim3(1), dim3(CG_T), 0, s, fvp, damping, residual_tol, n, x, r, p, p32, ax,
                       state, flag);
  }
  return hip_check(hipGetLastError(), "mrl_cg_update");
}

int mrl_cg_update_pack(const float* fvp, double damping, double residual_tol, int64_t n, double* x, double* r,
                       double* p, float* p32, double* ax, double* state, int32_t* flag, const mrl_mlp_desc* d,
                       float* image_t, void* stream) {
  if (!fvp || !x || !r || !p || !p32 || !state || !flag || !d || !image_t) return fail(E_ARG, "null pointer");
  if (!(MRL_CG_REG && n <= CG_SMALL_N && n <= 8 * CG_T))
    return fail(E_UNSUPPORTED, "mrl_cg_update_pack: the single-block register CG update only (n <= 8192)");
  const int64_t words = mrl_mlp_image_words_split(d);
  if (words < 0) return fail(E_UNSUPPORTED, "mrl_cg_update_pack: no split image for this net");
  if (mrl_mlp_num_params(d) != n) return fail(E_ARG, "mrl_cg_update_pack: n is not the net's parameter count");
  CgPack pk;
  pk.d = mlp_dims(d->n_in, d->n_out, d->head == MRL_HEAD_GAUSS);
  pk.b = bf16_dims(d->n_in, d->n_out);
  pk.image = image_t;
  hipLaunchKernelGGL((cg_update_reg_kernel<8, true>), dim3(1), dim3(CG_T), 0, (hipStream_t)stream, fvp, damping,
                     residual_tol, n, x, r, p, p32, ax, state, flag, pk);
  return hip_check(hipGetLastError(), "mrl_cg_update_pack");
}

int mrl_trpo_step(const float* fvp, const double* x, const float* g, double damping, double max_kl, int64_t n,
                  double* fullstep, double* out, void* stream) {
  if (!fvp || !x || !g || !fullstep || !out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(trpo_step_kernel, dim3(1), dim3(CG_T), 0, (hipStream_t)stream, fvp, x, g, damping, max_kl, n,
                     fullstep, out);
  return hip_check(hipGetLastError(), "mrl_trpo_step");
}

int mrl_trpo_step_ax(const double* ax, const double* x, const float* g, double max_kl, int64_t n, double* fullstep,
                     double* out, void* stream) {
  if (!ax || !x || !g || !fullstep || !out) return fail(E_ARG, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (n > CG_SMALL_N) {
    hipLaunchKernelGGL(cgm_step_part_kernel, dim3(CGB), dim3(CGB_T), 0, s, ax, x, g, n, out);
    hipLaunchKernelGGL(cgm_step_kernel, dim3(CGB), dim3(CGB_T), 0, s, x, max_kl, n, fullstep, out);
  } else {
    hipLaunchKernelGGL(trpo_step_ax_kernel, dim3(1), dim3(CG_T), 0, s, ax, x, g, max_kl, n, fullstep, out);
  }
  return hip_check(hipGetLastError(), "mrl_trpo_step_ax");
}

int mrl_axpy_cast(const float* theta_old, const double* fullstep, double frac, int64_t n, float* theta_out,
                  void* stream) {
  if (!theta_old || !fullstep || !theta_out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(axpy_cast_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, theta_old, fullstep, frac,
                     n, theta_out);
  return hip_check(hipGetLastError(), "mrl_axpy_cast");
}

int mrl_linesearch_candidates(const float* theta_old, const double* fullstep, int32_t k0, int32_t K, int64_t n,
                              float* out, void* stream) {
  if (!theta_old || !fullstep || !out) return fail(E_ARG, "null pointer");
  if (K <= 0 || k0 < 0 || k0 + K > 64) return fail(E_ARG, "mrl_linesearch_candidates: need 0 < K, 0 <= k0, k0 + K <= 64");
  hipLaunchKernelGGL(ls_candidates_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, theta_old, fullstep,
                     (int)k0, (int)K, n, out);
  return hip_check(hipGetLastError(), "mrl_linesearch_candidates");
}

int mrl_adam_step(float* theta, const float* g, float* m, float* v, double a_t, double beta1, double beta2,
                  double eps, int64_t n, void* stream) {
  if (!theta || !g || !m || !v) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, theta, g, m, v, (float)a_t,
                     (float)beta1, (float)beta2, (float)eps, n);
  return hip_check(hipGetLastError(), "mrl_adam_step");
}

int mrl_gather_rows(const void* src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst, void* stream) {
  if (!src || !idx || !dst) return fail(E_ARG, "null pointer");
  if (row_bytes <= 0 || row_bytes % 4 != 0) return fail(E_ARG, "row_bytes must be a positive multiple of 4");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * (row_bytes / 4))), dim3(256), 0, (hipStream_t)stream,
                     (const uint32_t*)src, idx, n, row_bytes / 4, (uint32_t*)dst);
  return hip_check(hipGetLastError(), "mrl_gather_rows");
}

int64_t mrl_moments_workspace_bytes(int64_t n) { return grid_for(n, 256, 1024) * 2 * (int64_t)sizeof(double); }

int mrl_moments_centered(const float* a, const float* b, int64_t n, const double* center, double* out,
                         void* workspace, void* stream) {
  if (!a || !out || !workspace) return fail(E_ARG, "null pointer");
  if (n <= 0) return fail(E_ARG, "mrl_moments: empty input");
  const int64_t g = grid_for(n, 256, 1024);
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(moments_kernel, dim3(g), dim3(256), 0, s, a, b, n, center, part);
  hipLaunchKernelGGL(moments_final_kernel, dim3(1), dim3(256), 0, s, part, g, (double)n, out);
  return hip_check(hipGetLastError(), "mrl_moments");
}

int mrl_moments(const float* a, const float* b, int64_t n, double* out, void* workspace, void* stream) {
  return mrl_moments_centered(a, b, n, nullptr, out, workspace, stream);
}

int64_t mrl_episode_stats_workspace_bytes(int64_t E) {
  return ((E + EPS_EB - 1) / EPS_EB) * 8 * (int64_t)sizeof(double);
}

int mrl_episode_stats(const float* rew, const uint8_t* flags, int64_t T, int64_t E, double* out, void* workspace,
                      void* stream) {
  if (!rew || !flags || !out || !workspace) return fail(E_ARG, "null pointer");
  if (T <= 0 || E <= 0) return fail(E_ARG, "mrl_episode_stats: empty batch");
  if ((int64_t)EPS_NC * 32 * (E + EPS_EB) >= ((int64_t)1 << 32))
    return fail(E_UNSUPPORTED, "mrl_episode_stats: E too large for 32-bit segment offsets");
  const int64_t nb = (E + EPS_EB - 1) / EPS_EB;
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  int L = 1;
  while (L < 32 && (int64_t)EPS_NC * L < T) L <<= 1;
#define MRL_EPS_LAUNCH(LL) \
  hipLaunchKernelGGL(episode_stats_kernel<LL>, dim3(nb), dim3(EPS_THREADS), 0, s, rew, flags, T, E, part)
  switch (L) {
    case 1: MRL_EPS_LAUNCH(1); break;
    case 2: MRL_EPS_LAUNCH(2); break;
    case 4: MRL_EPS_LAUNCH(4); break;
    case 8: MRL_EPS_LAUNCH(8); break;
    case 16: MRL_EPS_LAUNCH(16); break;
    default: MRL_EPS_LAUNCH(32); break;
  }
#undef MRL_EPS_LAUNCH
  hipLaunchKernelGGL(episode_stats_final_kernel, dim3(1), dim3(64), 0, s, part, nb, out);
  return hip_check(hipGetLastError(), "mrl_episode_stats");
}

int mrl_cast_scale_f32_f64(const float* in, double scale, int64_t n, double* out, void* stream) {
  if (!in || !out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(cast_scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, scale, n, out);
  return hip_check(hipGetLastError(), "mrl_cast_scale_f32_f64");
}

}  // extern "C"
