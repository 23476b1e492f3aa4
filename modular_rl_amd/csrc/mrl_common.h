// Shared device helpers for libmrl_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// v_mfma_f32_32x32x2_f32: exact f32 (a k-ordered fmaf chain), 64 cycles/SIMD.
// lane l supplies A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// D[i][j] lives in lane j (+32 for the upper row half), register r holds row
// i = (r&3) + 8*(r>>2) + 4*(l>>5).
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)
#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)
// v_mfma_f32_32x32x16_bf16 (bf16 operands, f32 accumulate; 32 cycles/SIMD, 16x the f32
// rate): lane l supplies A[i = l&31][k = 8(l>>5) + j] and B[k = 8(l>>5) + j][col l&31]
// in element j; the C/D layout is the f32 form's (cperm below).
#define MFMA32B(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)
// v_mfma_f32_16x16x32_bf16 (16 cycles/SIMD): lane l supplies A[i = l&15][k = 8(l>>4) + j]
// and B[k = 8(l>>4) + j][col l&15]; D[i][j] in lane j (+16 per row group), register r holds
// row i = 4(l>>4) + r (the 16x16x4 f32 form's layout)
#define MFMAB16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

namespace mrl {

// accumulator register r of lane half h -> row index inside a 32-row C tile
__host__ __device__ inline int cperm(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// The dispatcher deals consecutive block ids round-robin to the 8 XCDs (8 L2s).
// For kernels whose blocks own adjacent column segments of one row-major array,
// give each XCD a contiguous run of segments so a 128 B line shared by two
// neighbouring segments is fetched into one L2 only.  Identity unless nb % 8 == 0.
__device__ inline int64_t xcd_segment(int64_t b, int64_t nb) {
#ifdef MRL_NO_XCD_SEGMENT  // ablation build (tools/build_ablate.sh)
  (void)nb;
  return b;
#else
  return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
#endif
}

void set_error(const std::string& s);
int fail(int code, const std::string& s);
int hip_check(hipError_t e, const char* what);

enum { OK = 0, E_ARG = -1, E_UNSUPPORTED = -2, E_HIP = -3 };

// ------------------------------------------------------------------ Philox
// Bit-exact twin of oracle/philox.py.
struct u32x4 { uint32_t x, y, z, w; };

__device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}

__device__ inline double u01(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// two U[0,1) doubles for (seed, domain, gid, 64-bit word w, call)
__device__ inline void philox_uniform2(uint64_t seed, uint32_t domain, uint32_t gid, uint64_t w, uint32_t call,
                                       double& u0, double& u1) {
  const uint32_t k0 = (uint32_t)seed;
  const uint32_t k1 = (uint32_t)(seed >> 32) ^ (uint32_t)(0x9E3779B9u * domain);
  const u32x4 r = philox4x32_10(u32x4{gid, (uint32_t)w, (uint32_t)(w >> 32), call}, k0, k1);
  u0 = u01(r.x, r.y);
  u1 = u01(r.z, r.w);
}

}  // namespace mrl
