// Diagnostic: dependent-chain latency (shader cycles per link, one wave) of the fp64
// operations on the rollout's serial chain -- fma, the compiler's IEEE division and
// sqrt, and the division's pieces -- on gfx950 (the loop unrolled by 8: per-link figures
// are the chain's own latency).  hipcc --offload-arch=gfx950 -O3
// tools/fp64_latency.hip -o tools/var/fp64_latency && tools/var/fp64_latency
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 256;

template <int OP>
__global__ void chain(const double* in, double* out, long long* cyc) {
  double x = in[threadIdx.x];
  const double c = in[64 + threadIdx.x];
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < N; ++i) {
    if constexpr (OP == 0) x = __builtin_fma(x, c, 0.25);          // one v_fma_f64
    if constexpr (OP == 1) x = 1.0 / (x + c);                       // add + IEEE division
    if constexpr (OP == 2) x = __builtin_sqrt(x + c);               // add + IEEE sqrt
    if constexpr (OP == 3) x = x + c;                               // one v_add_f64
    if constexpr (OP == 4) x = __builtin_amdgcn_rcp(x + c);         // add + v_rcp_f64
    if constexpr (OP == 5) {                                        // add + rcp + 2 Newton + 1 correction
      const double d = x + c;
      double r = __builtin_amdgcn_rcp(d);
      double e = __builtin_fma(-d, r, 1.0);
      r = __builtin_fma(r, e, r);
      e = __builtin_fma(-d, r, 1.0);
      r = __builtin_fma(r, e, r);
      const double rem = __builtin_fma(-d, r, 1.0);
      x = __builtin_fma(rem, r, r);
    }
    if constexpr (OP == 6) x = (x * c) / 3.0;                       // mul + division by a constant
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double h[128];
  for (int i = 0; i < 64; ++i) {
    h[i] = 1.0 + i * 1e-3;
    h[64 + i] = 0.5 + i * 1e-4;
  }
  double *in, *out;
  long long* cyc;
  hipMalloc(&in, sizeof h);
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&cyc, sizeof(long long));
  hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
  const char* names[] = {"fma_f64", "add+div_f64", "add+sqrt_f64", "add_f64", "add+rcp_f64", "add+rcp+newton2+corr",
                         "mul+div_by_const"};
  for (int op = 0; op < 7; ++op) {
    long long best = 1LL << 60;
    for (int rep = 0; rep < 5; ++rep) {
      switch (op) {
        case 0: chain<0><<<1, 64>>>(in, out, cyc); break;
        case 1: chain<1><<<1, 64>>>(in, out, cyc); break;
        case 2: chain<2><<<1, 64>>>(in, out, cyc); break;
        case 3: chain<3><<<1, 64>>>(in, out, cyc); break;
        case 4: chain<4><<<1, 64>>>(in, out, cyc); break;
        case 5: chain<5><<<1, 64>>>(in, out, cyc); break;
        case 6: chain<6><<<1, 64>>>(in, out, cyc); break;
      }
      long long c;
      hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    printf("%-24s %7.1f cycles per link\n", names[op], (double)best / N);
  }
  return 0;
}
