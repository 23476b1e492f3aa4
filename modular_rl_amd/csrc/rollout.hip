// Batched lock-step rollout: E envs per GPU advance one step per launch.
//
// Replaces the reference's serial per-step loop (core.py:182-221):
//     ob = agent.obfilt(ob)                 ZFilter, filters.py:30-38
//     action, {"prob"} = agent.act(ob)      StochPolicy.act, core.py:261-267
//     ob, rew, done, _ = env.step(action)   gym
//     agent.rewfilt(rew)                    stats only, core.py:198-199
// Per launch (step t) every block
//   1. merges the per-block Welford partials of the E raw observations of step t
//      (and rewards of step t-1) -- published by launch t-1 -- into the running
//      stat, in block order (so every block derives the identical state; block 0
//      stores it; ping-pong buffers by step parity),
//   2. normalises its envs' observations (x - mean)/(std + 1e-8), clip +-5, stores
//      them as the trajectory rows (fp32) and in LDS,
//   3. runs the policy MLP forward on MFMA (32 envs per wave, image in LDS),
//   4. samples the action (Philox counter stream or injected noise),
//   5. steps the env (fp64), auto-resets finished episodes, writes reward/flags,
//   6. publishes the block's Welford partial of the new raw obs and the reward.
#include <math.h>

#include "../../include/mrl_hip.h"
#include "envs.h"
#include "mlp_device.h"

namespace mrl {

constexpr int RB = 256;          // threads per block
constexpr int ENVS_PER_BLOCK = 128;
constexpr int MAXD = 16;         // obs dims + 1 (reward)

struct EnvInfo {
  int ns, obs, act, discrete, max_steps;
};
__host__ __device__ inline EnvInfo env_info(int id) {
  if (id == MRL_ENV_CARTPOLE) return EnvInfo{CP_NS, CP_OBS, 2, 1, 200};
  return EnvInfo{HP_NS, HP_OBS, HP_ACT, 0, 1000};
}
__host__ __device__ inline int filt_doubles(int obs) { return 2 + 2 * (obs + 1); }

__device__ inline void env_reset(int id, const double* u, double* s) {
  if (id == MRL_ENV_CARTPOLE) cartpole_reset(u, s);
  else hopper_reset(u, s);
}
__device__ inline void env_obs(int id, const double* s, double* o) {
  if (id == MRL_ENV_CARTPOLE) cartpole_obs(s, o);
  else hopper_obs(s, o);
}

struct RollArgs {
  mrl_rollout_desc d;
  mrl_rollout_bufs b;
  EnvInfo ei;
  int nb;      // blocks
  int FS, RS;  // filter / record doubles
};

// reset-noise uniforms for one env: (gid, episode counter) on domain 1
__device__ inline void reset_env(const RollArgs& a, int e, double* s) {
  const int E = a.d.n_envs;
  const uint32_t gid = (uint32_t)(a.d.env_offset + e);
  const uint64_t w = (uint64_t)(uint32_t)a.b.env_int[E + e];
  double u[HP_NS];
  const int nu = a.ei.discrete ? 4 : 12;
  for (int c = 0; c < nu / 2; ++c) philox_uniform2(a.d.seed, 1, gid, w, (uint32_t)c, u[2 * c], u[2 * c + 1]);
  env_reset(a.d.env_id, u, s);
  a.b.env_int[E + e] = (int32_t)(w + 1);
  a.b.env_int[e] = 0;
}

// sum over the 16 lanes of an aligned 16-lane group (fixed butterfly order)
__device__ inline double sum16(double v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// per-block two-pass (mean, M2) partial of vals[ENVS_PER_BLOCK][D] (doubles in LDS):
// thread (k = tid/16, j = tid%16) covers envs j, j+16, ...; 16-lane butterflies.
__device__ inline void publish_partial(const RollArgs& a, const double* vals, int nvalid, int D, bool with_rew,
                                       double* rec_out) {
  const int k = threadIdx.x >> 4, j = threadIdx.x & 15;
  double s = 0.0;
  if (k < D)
    for (int i = j; i < nvalid; i += 16) s += vals[i * D + k];
  const double mean = nvalid > 0 ? sum16(s) / (double)nvalid : 0.0;
  double m2 = 0.0;
  if (k < D)
    for (int i = j; i < nvalid; i += 16) {
      const double dv = vals[i * D + k] - mean;
      m2 += dv * dv;
    }
  m2 = sum16(m2);
  if (k < D && j == 0) {
    double* r = rec_out + (int64_t)blockIdx.x * a.RS;
    r[2 + k] = mean;
    r[2 + D + k] = m2;
    if (k == 0) {
      r[0] = (double)nvalid;
      r[1] = with_rew ? (double)nvalid : 0.0;
    }
  }
}

// combine the per-block records of one column k into a batch (n, mean, M2):
// mean = sum n_b mean_b / n ; M2 = sum (M2_b + n_b (mean_b - mean)^2).
// Called by all 16 lanes of thread group k; every lane returns the same values.
__device__ inline void batch_of_records(const double* rec, int nb, int RS, int D, int O, int k, int j, double& bn,
                                        double& bm, double& bs) {
  const bool isr = (k == O);
  double n = 0.0, sm = 0.0;
  for (int b = j; b < nb; b += 16) {
    const double* r = rec + (int64_t)b * RS;
    const double nb_ = r[isr ? 1 : 0];
    n += nb_;
    sm += nb_ * r[2 + k];
  }
  n = sum16(n);
  sm = sum16(sm);
  const double mean = n > 0.0 ? sm / n : 0.0;
  double m2 = 0.0;
  for (int b = j; b < nb; b += 16) {
    const double* r = rec + (int64_t)b * RS;
    const double nb_ = r[isr ? 1 : 0];
    if (nb_ > 0.0) {
      const double dm = r[2 + k] - mean;
      m2 += r[2 + D + k] + nb_ * dm * dm;
    }
  }
  bn = n;
  bm = mean;
  bs = sum16(m2);
}

// Chan merge of (nb, mb, m2b) into (n, M, S); for nb == 1 this is RunningStat.push
__device__ inline void chan_merge(double& n, double& M, double& S, double nb, double mb, double m2b) {
  if (nb <= 0.0) return;
  const double na = n;
  const double nn = na + nb;
  const double delta = mb - M;
  const double newM = M + (delta * nb) / nn;
  S = S + m2b + delta * (mb - newM) * nb;
  M = newM;
  n = nn;
}

__global__ __launch_bounds__(RB) void rollout_reset_kernel(RollArgs a) {
  __shared__ double vals[ENVS_PER_BLOCK * MAXD];
  const int E = a.d.n_envs, O = a.ei.obs, D = O + 1;
  const int le = threadIdx.x;
  const int e = blockIdx.x * ENVS_PER_BLOCK + le;
  if (le < ENVS_PER_BLOCK && e < E) {
    double s[HP_NS], o[HP_OBS];
    reset_env(a, e, s);
    for (int i = 0; i < a.ei.ns; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
    env_obs(a.d.env_id, s, o);
    for (int k = 0; k < O; ++k) vals[le * D + k] = o[k];
    vals[le * D + O] = 0.0;
  }
  __syncthreads();
  const int nvalid = min(ENVS_PER_BLOCK, E - (int)blockIdx.x * ENVS_PER_BLOCK);
  publish_partial(a, vals, nvalid, D, false, a.b.records);
}

__global__ __launch_bounds__(RB) void rollout_step_kernel(RollArgs a, MlpDims md, const float* __restrict__ theta,
                                                          const float* __restrict__ img, int t) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double vals[ENVS_PER_BLOCK * MAXD];
  __shared__ double fmean[MAXD], fden[MAXD];
  __shared__ float xt[4][32][MAX_IN];

  const int E = a.d.n_envs, O = a.ei.obs, D = O + 1, A = md.A;
  for (int i = threadIdx.x; i < md.fwd_size / 4; i += RB)
    reinterpret_cast<float4*>(lds)[i] = reinterpret_cast<const float4*>(img)[i];

  // 1. running-stat merge (filters.py:30-31 push, per step over all envs)
  const double* fs_in = a.b.filter_state + (t & 1) * a.FS;
  double* fs_out = a.b.filter_state + ((t + 1) & 1) * a.FS;
  const double* rec_in = a.b.records + (int64_t)(t & 1) * a.nb * a.RS;
  double* rec_out = a.b.records + (int64_t)((t + 1) & 1) * a.nb * a.RS;
  if ((int)(threadIdx.x >> 4) < D) {
    const int k = threadIdx.x >> 4, j = threadIdx.x & 15;
    const bool isr = (k == O);
    double n = fs_in[isr ? 1 : 0], M = fs_in[2 + k], S = fs_in[2 + D + k];
    // combine the block partials into one batch, then one Chan merge into the stat
    double bn, bm, bs;
    batch_of_records(rec_in, a.nb, a.RS, D, O, k, j, bn, bm, bs);
    chan_merge(n, M, S, bn, bm, bs);
    if (j != 0) {
    } else if (blockIdx.x == 0) {
      if (k == 0) fs_out[0] = n;
      if (isr) fs_out[1] = n;
      fs_out[2 + k] = M;
      fs_out[2 + D + k] = S;
    }
    if (!isr && j == 0) {
      const double var = n > 1.0 ? S / (n - 1.0) : M * M;  // running_stat.py:27
      fmean[k] = M;
      fden[k] = sqrt(var) + 1e-8;
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int le = wave * 32 + j;
  const int e = blockIdx.x * ENVS_PER_BLOCK + le;
  const bool valid = e < E;
  const int64_t row = (int64_t)t * E + e;
  double s[HP_NS];
  if (valid)
    for (int i = 0; i < a.ei.ns; ++i) s[i] = a.b.env_state[(int64_t)i * E + e];

  // 2. filtered observation (core.py:191-192)
  if (valid) {
    double o[HP_OBS];
    env_obs(a.d.env_id, s, o);
    for (int k = 0; k < O; ++k) {
      double v = o[k];
      if (a.d.filter) {
        v = v - fmean[k];
        v = v / fden[k];
        v = v < -5.0 ? -5.0 : (v > 5.0 ? 5.0 : v);
      }
      const float vf = (float)v;
      if (h == 0) a.b.obs[row * O + k] = vf;
      xt[wave][j][k] = vf;
    }
  }
  WAVE_LDS_ORDER();

  // 3. policy forward
  struct XL {
    const float* p;
    int O;
    bool valid;
    __device__ inline float operator()(int k) const { return (valid && k < O) ? p[k] : 0.f; }
  } xl{&xt[wave][j][0], O, valid};
  float z[MAX_OUT];
  forward_head_lowreg(lds, md, xl, lane, z);

  bool done = false, last = false, term = false;
  double rew = 0.0;
  if (valid && h == 0) {
    const uint32_t gid = (uint32_t)(a.d.env_offset + e);
    const uint64_t w = (uint64_t)(*a.b.iteration) * (uint64_t)a.d.horizon + (uint64_t)t;
    // 4. sample (core.py:261-267; distributions.py:3-13 / core.py:432-435)
    if (a.ei.discrete) {
      float m = z[0];
      for (int q = 1; q < A; ++q) m = fmaxf(m, z[q]);
      float p[MAX_OUT], se = 0.f;
      for (int q = 0; q < A; ++q) { p[q] = expf(z[q] - m); se += p[q]; }
      for (int q = 0; q < A; ++q) p[q] = p[q] / se;
      double u, u1;
      if (a.b.noise != nullptr) u = reinterpret_cast<const double*>(a.b.noise)[row];
      else philox_uniform2(a.d.seed, 0, gid, w, 0, u, u1);
      int act = 0;
      float cs = 0.f;
      for (int q = 0; q < A; ++q) {
        cs += p[q];
        if ((double)cs > u) { act = q; break; }
      }
      reinterpret_cast<int32_t*>(a.b.act)[row] = act;
      for (int q = 0; q < A; ++q) a.b.prob[row * A + q] = p[q];
      cartpole_step(s, act, rew, done);
    } else {
      const float* logstd = theta + md.tls;
      float av[MAX_OUT];
      double zn[MAX_OUT + 1];
      if (a.b.noise != nullptr) {
        for (int q = 0; q < A; ++q) zn[q] = reinterpret_cast<const double*>(a.b.noise)[row * A + q];
      } else {
        for (int c = 0; c < (A + 1) / 2; ++c) {
          double u0, u1;
          philox_uniform2(a.d.seed, 0, gid, w, (uint32_t)c, u0, u1);
          const double rad = sqrt(-2.0 * log(1.0 - u0));
          const double ang = 2.0 * 3.141592653589793 * u1;
          zn[2 * c] = rad * cos(ang);
          zn[2 * c + 1] = rad * sin(ang);
        }
      }
      for (int q = 0; q < A; ++q) {
        const float sd = expf(logstd[q]);
        av[q] = __fadd_rn(__fmul_rn((float)zn[q], sd), z[q]);
        reinterpret_cast<float*>(a.b.act)[row * A + q] = av[q];
        a.b.prob[row * 2 * A + q] = z[q];
        a.b.prob[row * 2 * A + A + q] = sd;
      }
      hopper_step(s, av, rew, done);
    }
    // 5. episode bookkeeping: gym TimeLimit => done (terminated, bootstrap 0);
    //    the rollout loop limit / horizon cut => not terminated (core.py:190-207, 73)
    const int ept = a.b.env_int[e];
    a.b.ep_t[row] = ept;
    term = done || (ept + 1 >= a.ei.max_steps);
    last = term || (ept + 1 >= a.d.timestep_limit) || (t == a.d.horizon - 1);
    a.b.rew[row] = (float)rew;
    a.b.flags[row] = (uint8_t)((last ? 1 : 0) | (term ? 2 : 0));
    if (last && t < a.d.horizon - 1) reset_env(a, e, s);
    else a.b.env_int[e] = ept + 1;
    for (int i = 0; i < a.ei.ns; ++i) a.b.env_state[(int64_t)i * E + e] = s[i];
    // 6. raw next observation + reward into the block partial
    double o[HP_OBS];
    env_obs(a.d.env_id, s, o);
    for (int k = 0; k < O; ++k) vals[le * D + k] = o[k];
    vals[le * D + O] = rew;
  }
  __syncthreads();
  const int nvalid = min(ENVS_PER_BLOCK, E - (int)blockIdx.x * ENVS_PER_BLOCK);
  publish_partial(a, vals, nvalid, D, true, rec_out);
}

__global__ void rollout_finish_kernel(RollArgs a) {
  const int O = a.ei.obs, D = O + 1, T = a.d.horizon;
  const double* fs_in = a.b.filter_state + (T & 1) * a.FS;
  double* fs_out = a.b.filter_state;
  const double* rec_in = a.b.records + (int64_t)(T & 1) * a.nb * a.RS;
  const int k = threadIdx.x >> 4, j = threadIdx.x & 15;
  const bool isr = (k == O);
  double n = 0.0, M = 0.0, S = 0.0;
  if (k < D) {
    n = fs_in[isr ? 1 : 0];
    M = fs_in[2 + k];
    S = fs_in[2 + D + k];
    if (isr) {  // the last step's rewards still go through rewfilt (core.py:199)
      double bn, bm, bs;
      batch_of_records(rec_in, a.nb, a.RS, D, O, k, j, bn, bm, bs);
      chan_merge(n, M, S, bn, bm, bs);
    }
  }
  __syncthreads();  // fs_in may alias fs_out (T even)
  if (k < D && j == 0) {
    if (k == 0) fs_out[0] = n;
    if (isr) fs_out[1] = n;
    fs_out[2 + k] = M;
    fs_out[2 + D + k] = S;
  }
  if (k == 0) *a.b.iteration += 1;
}

}  // namespace mrl

using namespace mrl;

static int check_roll(const mrl_rollout_desc* d, const mrl_rollout_bufs* b) {
  if (!d || !b) return fail(E_ARG, "null desc/bufs");
  if (d->env_id != MRL_ENV_CARTPOLE && d->env_id != MRL_ENV_HOPPER) return fail(E_UNSUPPORTED, "unknown env_id");
  if (d->n_envs <= 0 || d->horizon <= 0 || d->timestep_limit <= 0) return fail(E_ARG, "bad sizes");
  if (!b->env_state || !b->env_int || !b->filter_state || !b->records || !b->iteration) return fail(E_ARG, "null state");
  return OK;
}

static RollArgs make_args(const mrl_rollout_desc* d, const mrl_rollout_bufs* b) {
  RollArgs a;
  a.d = *d;
  a.b = *b;
  a.ei = env_info(d->env_id);
  a.nb = (d->n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  a.FS = filt_doubles(a.ei.obs);
  a.RS = a.FS;
  return a;
}

extern "C" {

int64_t mrl_env_state_doubles(int32_t env_id) { return env_info(env_id).ns; }
int64_t mrl_filter_doubles(int32_t env_id) { return filt_doubles(env_info(env_id).obs); }
int64_t mrl_record_doubles(int32_t env_id) { return filt_doubles(env_info(env_id).obs); }
int64_t mrl_rollout_blocks(int32_t n_envs) { return (n_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK; }

int mrl_rollout_reset(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  RollArgs a = make_args(d, b);
  hipLaunchKernelGGL(rollout_reset_kernel, dim3(a.nb), dim3(RB), 0, (hipStream_t)stream, a);
  return hip_check(hipGetLastError(), "mrl_rollout_reset");
}

int mrl_rollout_step(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, const float* image,
                     const mrl_rollout_bufs* b, int32_t t, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  if (!pol || !theta || !image) return fail(E_ARG, "null policy");
  if (!b->obs || !b->act || !b->prob || !b->rew || !b->flags || !b->ep_t) return fail(E_ARG, "null trajectory buffer");
  EnvInfo ei = env_info(d->env_id);
  const bool gauss = pol->head == MRL_HEAD_GAUSS;
  if (pol->n_in != ei.obs || pol->n_out != ei.act || gauss == (bool)ei.discrete || pol->n_hidden != HID ||
      pol->n_layers != 2)
    return fail(E_ARG, "policy shape does not match the env");
  if (t < 0 || t >= d->horizon) return fail(E_ARG, "t out of range");
  RollArgs a = make_args(d, b);
  MlpDims md = mlp_dims(pol->n_in, pol->n_out, gauss);
  size_t shm = (size_t)md.fwd_size * 4;
  hipLaunchKernelGGL(rollout_step_kernel, dim3(a.nb), dim3(RB), shm, (hipStream_t)stream, a, md, theta, image, t);
  return hip_check(hipGetLastError(), "mrl_rollout_step");
}

int mrl_rollout_finish(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream) {
  int rc = check_roll(d, b);
  if (rc) return rc;
  RollArgs a = make_args(d, b);
  hipLaunchKernelGGL(rollout_finish_kernel, dim3(1), dim3(RB), 0, (hipStream_t)stream, a);
  return hip_check(hipGetLastError(), "mrl_rollout_finish");
}

}  // extern "C"
