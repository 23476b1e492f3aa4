// Advantage scan, standardisation and the device-resident CG / step-scaling /
// line-search vector kernels of the TRPO update.
//
// GAE (core.py:63-75 + misc_utils.py:9-27 `discount` via scipy lfilter): on
// time-major [T, E] rows the per-path reverse recurrences
//     adv_t = delta_t + gamma*lam*cont_t*adv_{t+1},  ret_t = r_t + gamma*cont_t*ret_{t+1}
// are linear, so each (chunk of L steps, env) is summarised as an affine map
// (A, B): adv_in = A + B*adv_out.  Pass 1 writes the summaries; pass 2 folds the
// summaries of later chunks into a carry and re-scans its chunk (the second read
// of r/v/flags is served by the 256 MiB Infinity Cache at the benchmark size).
// Scans run in fp64 like lfilter; outputs are fp32.
#include <math.h>

#include "../../include/mrl_hip.h"
#include "mrl_common.h"

namespace mrl {

constexpr int GAE_CHUNK = 32;

struct Summ {
  double A, B, R, C;
};

__device__ inline double delta_at(const float* rew, const float* v, const uint8_t* flags, int64_t t, int64_t T,
                                  int64_t E, int64_t e, double gamma, bool& cont) {
  const int64_t i = t * E + e;
  const uint8_t fl = flags[i];
  cont = !(fl & 1) && (t + 1 < T);
  const double vt = (double)v[i];
  // bootstrap b1[t+1]: next baseline inside the episode, 0 if terminated, else b[-1] (core.py:73)
  const double boot = cont ? (double)v[i + E] : ((fl & 2) ? 0.0 : vt);
  return (double)rew[i] + gamma * boot - vt;
}

__global__ void gae_summary_kernel(const float* __restrict__ rew, const float* __restrict__ v,
                                   const uint8_t* __restrict__ flags, int64_t T, int64_t E, double gamma, double lam,
                                   Summ* __restrict__ summ) {
  const int64_t C = (T + GAE_CHUNK - 1) / GAE_CHUNK;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= C * E) return;
  const int64_t c = id / E, e = id % E;
  const int64_t t0 = c * GAE_CHUNK, t1 = min(T, t0 + GAE_CHUNK);
  double A = 0.0, B = 1.0, R = 0.0, Cc = 1.0;
  const double gl = gamma * lam;
  for (int64_t t = t1 - 1; t >= t0; --t) {
    bool cont;
    const double d = delta_at(rew, v, flags, t, T, E, e, gamma, cont);
    const double k = cont ? 1.0 : 0.0;
    A = d + gl * k * A;
    B = gl * k * B;
    R = (double)rew[t * E + e] + gamma * k * R;
    Cc = gamma * k * Cc;
  }
  summ[id] = Summ{A, B, R, Cc};
}

__global__ void gae_final_kernel(const float* __restrict__ rew, const float* __restrict__ v,
                                 const uint8_t* __restrict__ flags, int64_t T, int64_t E, double gamma, double lam,
                                 const Summ* __restrict__ summ, float* __restrict__ adv, float* __restrict__ ret,
                                 double* __restrict__ part) {
  __shared__ double red[2][256];
  const int64_t C = (T + GAE_CHUNK - 1) / GAE_CHUNK;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (id < C * E) {
    const int64_t c = id / E, e = id % E;
    double a = 0.0, r = 0.0;
    for (int64_t cc = C - 1; cc > c; --cc) {
      const Summ s = summ[cc * E + e];
      a = s.A + s.B * a;
      r = s.R + s.C * r;
    }
    const int64_t t0 = c * GAE_CHUNK, t1 = min(T, t0 + GAE_CHUNK);
    const double gl = gamma * lam;
    for (int64_t t = t1 - 1; t >= t0; --t) {
      bool cont;
      const double d = delta_at(rew, v, flags, t, T, E, e, gamma, cont);
      const double k = cont ? 1.0 : 0.0;
      a = d + gl * k * a;
      r = (double)rew[t * E + e] + gamma * k * r;
      const float af = (float)a;
      adv[t * E + e] = af;
      ret[t * E + e] = (float)r;
      s1 += (double)af;
      s2 += (double)af * (double)af;
    }
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
    part[blockIdx.x * 2 + 0] = red[0][0];
    part[blockIdx.x * 2 + 1] = red[1][0];
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

__global__ void standardize_kernel(float* __restrict__ adv, int64_t n, const double* __restrict__ mom) {
  const double cnt = mom[2];
  const double mean = mom[0] / cnt;
  const double var = fmax(mom[1] / cnt - mean * mean, 0.0);
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

__device__ inline double block_sum(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = CG_T / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(CG_T) void cg_init_kernel(const double* __restrict__ b, int64_t n, double* x, double* r,
                                                       double* p, float* p32, double* state, int32_t* flag) {
  __shared__ double red[CG_T];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += CG_T) {
    const double bi = b[i];
    x[i] = 0.0;
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
                                                         double* state, int32_t* flag) {
  __shared__ double red[CG_T];
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

__global__ __launch_bounds__(CG_T) void trpo_step_kernel(const float* __restrict__ fvp, const double* __restrict__ x,
                                                         const float* __restrict__ g, double damping, double max_kl,
                                                         int64_t n, double* fullstep, double* out) {
  __shared__ double red[CG_T];
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

__global__ void axpy_cast_kernel(const float* __restrict__ a, const double* __restrict__ b, double frac, int64_t n,
                                 float* __restrict__ o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = (float)((double)a[i] + frac * b[i]);
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
// per-block fp64 (sum, sumsq) of (a - b) -> part[block][2]
__global__ void moments_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                               double* __restrict__ part) {
  __shared__ double red[2][256];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = (double)a[i] - (b ? (double)b[i] : 0.0);
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

// episode statistics over time-major rows (core.py:31-44): one thread per env scans
// its rows in time order; part[block][8] = (n_ep, sum R, sum R^2, max R, sum L, max L, sum r, 0)
__global__ void episode_stats_kernel(const float* __restrict__ rew, const uint8_t* __restrict__ flags, int64_t T,
                                     int64_t E, double* __restrict__ part) {
  __shared__ double red[6][256];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double cnt = 0, sr = 0, sr2 = 0, mr = -INFINITY, sl = 0, ml = 0;
  if (e < E) {
    double ep = 0.0, len = 0.0;
    for (int64_t t = 0; t < T; ++t) {
      ep += (double)rew[t * E + e];
      len += 1.0;
      if (flags[t * E + e] & 1) {
        cnt += 1.0;
        sr += ep;
        sr2 += ep * ep;
        mr = fmax(mr, ep);
        sl += len;
        ml = fmax(ml, len);
        ep = 0.0;
        len = 0.0;
      }
    }
  }
  red[0][threadIdx.x] = cnt;
  red[1][threadIdx.x] = sr;
  red[2][threadIdx.x] = sr2;
  red[3][threadIdx.x] = mr;
  red[4][threadIdx.x] = sl;
  red[5][threadIdx.x] = ml;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      for (int q = 0; q < 6; ++q) {
        if (q == 3 || q == 5) red[q][threadIdx.x] = fmax(red[q][threadIdx.x], red[q][threadIdx.x + o]);
        else red[q][threadIdx.x] += red[q][threadIdx.x + o];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[blockIdx.x * 8 + threadIdx.x] = red[threadIdx.x][0];
  if (threadIdx.x == 6) part[blockIdx.x * 8 + 6] = 0.0;
  if (threadIdx.x == 7) part[blockIdx.x * 8 + 7] = 0.0;
}

__global__ void episode_stats_final_kernel(const double* __restrict__ part, int64_t nb, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double a[6] = {0, 0, 0, -INFINITY, 0, 0};
  for (int64_t b = 0; b < nb; ++b) {
    for (int q = 0; q < 6; ++q) {
      const double v = part[b * 8 + q];
      a[q] = (q == 3 || q == 5) ? fmax(a[q], v) : a[q] + v;
    }
  }
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

int64_t mrl_gae_workspace_bytes(int64_t T, int64_t E) {
  const int64_t C = (T + GAE_CHUNK - 1) / GAE_CHUNK;
  const int64_t nb = (C * E + 255) / 256;
  return C * E * (int64_t)sizeof(Summ) + nb * 2 * (int64_t)sizeof(double) + 64;
}

int mrl_gae(const float* rew, const float* vpred, const uint8_t* flags, int64_t T, int64_t E, double gamma, double lam,
            float* adv, float* ret, double* moments, void* workspace, void* stream) {
  if (!rew || !vpred || !flags || !adv || !ret || !moments || !workspace) return fail(E_ARG, "null pointer");
  if (T <= 0 || E <= 0) return OK;
  const int64_t C = (T + GAE_CHUNK - 1) / GAE_CHUNK;
  const int64_t nthreads = C * E;
  const int64_t nb = (nthreads + 255) / 256;
  Summ* summ = reinterpret_cast<Summ*>(workspace);
  double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + C * E * sizeof(Summ));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gae_summary_kernel, dim3(nb), dim3(256), 0, s, rew, vpred, flags, T, E, gamma, lam, summ);
  hipLaunchKernelGGL(gae_final_kernel, dim3(nb), dim3(256), 0, s, rew, vpred, flags, T, E, gamma, lam, summ, adv, ret,
                     part);
  hipLaunchKernelGGL(moments_final_kernel, dim3(1), dim3(256), 0, s, part, nb, (double)(T * E), moments);
  return hip_check(hipGetLastError(), "mrl_gae");
}

int mrl_standardize(float* adv, int64_t n, const double* moments, void* stream) {
  if (!adv || !moments) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(standardize_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, adv, n, moments);
  return hip_check(hipGetLastError(), "mrl_standardize");
}

int mrl_vf_target(const float* ret, const float* vpred, double mixfrac, int64_t n, float* y, void* stream) {
  if (!ret || !vpred || !y) return fail(E_ARG, "null pointer");
  if (n <= 0) return OK;
  hipLaunchKernelGGL(vf_target_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, ret, vpred, mixfrac, n, y);
  return hip_check(hipGetLastError(), "mrl_vf_target");
}

int mrl_cg_init(const double* b, int64_t n, double* x, double* r, double* p, float* p32, double* state, int32_t* flag,
                void* stream) {
  if (!b || !x || !r || !p || !p32 || !state || !flag) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(cg_init_kernel, dim3(1), dim3(CG_T), 0, (hipStream_t)stream, b, n, x, r, p, p32, state, flag);
  return hip_check(hipGetLastError(), "mrl_cg_init");
}

int mrl_cg_update(const float* fvp, double damping, double residual_tol, int64_t n, double* x, double* r, double* p,
                  float* p32, double* state, int32_t* flag, void* stream) {
  if (!fvp || !x || !r || !p || !p32 || !state || !flag) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(cg_update_kernel, dim3(1), dim3(CG_T), 0, (hipStream_t)stream, fvp, damping, residual_tol, n, x, r,
                     p, p32, state, flag);
  return hip_check(hipGetLastError(), "mrl_cg_update");
}

int mrl_trpo_step(const float* fvp, const double* x, const float* g, double damping, double max_kl, int64_t n,
                  double* fullstep, double* out, void* stream) {
  if (!fvp || !x || !g || !fullstep || !out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(trpo_step_kernel, dim3(1), dim3(CG_T), 0, (hipStream_t)stream, fvp, x, g, damping, max_kl, n,
                     fullstep, out);
  return hip_check(hipGetLastError(), "mrl_trpo_step");
}

int mrl_axpy_cast(const float* theta_old, const double* fullstep, double frac, int64_t n, float* theta_out,
                  void* stream) {
  if (!theta_old || !fullstep || !theta_out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(axpy_cast_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, theta_old, fullstep, frac,
                     n, theta_out);
  return hip_check(hipGetLastError(), "mrl_axpy_cast");
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

int mrl_moments(const float* a, const float* b, int64_t n, double* out, void* workspace, void* stream) {
  if (!a || !out || !workspace) return fail(E_ARG, "null pointer");
  const int64_t g = grid_for(n, 256, 1024);
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(moments_kernel, dim3(g), dim3(256), 0, s, a, b, n, part);
  hipLaunchKernelGGL(moments_final_kernel, dim3(1), dim3(256), 0, s, part, g, (double)n, out);
  return hip_check(hipGetLastError(), "mrl_moments");
}

int64_t mrl_episode_stats_workspace_bytes(int64_t E) { return ((E + 255) / 256) * 8 * (int64_t)sizeof(double); }

int mrl_episode_stats(const float* rew, const uint8_t* flags, int64_t T, int64_t E, double* out, void* workspace,
                      void* stream) {
  if (!rew || !flags || !out || !workspace) return fail(E_ARG, "null pointer");
  const int64_t nb = (E + 255) / 256;
  double* part = reinterpret_cast<double*>(workspace);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(episode_stats_kernel, dim3(nb), dim3(256), 0, s, rew, flags, T, E, part);
  hipLaunchKernelGGL(episode_stats_final_kernel, dim3(1), dim3(64), 0, s, part, nb, out);
  return hip_check(hipGetLastError(), "mrl_episode_stats");
}

int mrl_cast_scale_f32_f64(const float* in, double scale, int64_t n, double* out, void* stream) {
  if (!in || !out) return fail(E_ARG, "null pointer");
  hipLaunchKernelGGL(cast_scale_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, scale, n, out);
  return hip_check(hipGetLastError(), "mrl_cast_scale_f32_f64");
}

}  // extern "C"
