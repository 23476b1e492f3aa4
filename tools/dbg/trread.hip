// Diagnostic: what ds_read_b64_tr_b16 returns per lane for given per-lane addresses.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)i;  // value = row*64 + col
  __syncthreads();
  const int lane = threadIdx.x, G = lane >> 4;
  int q, p;
  if (mode == 0) { q = (lane >> 2) & 3; p = lane & 3; } else { q = lane & 3; p = (lane >> 2) & 3; }
  const short* a = lds + (4 * G + q) * 64 + 4 * p;
  typedef __attribute__((address_space(3))) s16x4 L;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L*)a);
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d, mode);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d (value = row*64 + col)\n", mode);
    for (int l = 0; l < 20; ++l) printf(" lane %2d: %4d %4d %4d %4d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
  }
  return 0;
}
