// Per-row epilogues shared by the fused 64-wide rows kernel (mlp_kernels.hip) and the
// layered-path head kernel (gemm.hip): given the head pre-activation z (and its
// tangent dz for the Fisher product) of one row, produce prob rows, the surrogate /
// KL / entropy partial sums, the head-gradient row, or the VF squared error.
#pragma once
#include "../../include/mrl_hip.h"
#include "mlp_layout.h"

namespace mrl {

struct RowsArgs {
  MlpDims d;
  int head, n_obs, gh, A;
  const float* x;
  const int32_t* ept;
  double ts_limit;
  int64_t n;
  double inv_ng;
  const void* act;
  const float* adv;
  const float* oldprob;
  const float* target;
  float* out;
  float* ghead;
  double* partial;
  const float* logstd;   // theta + tls (DiagGauss) or nullptr
  const float* dlogstd;  // tangent + tls (EPI_FVP, DiagGauss) or nullptr
  // PPO (ppo.py:3-229): pensurr = surr + c_kl * kl + cutoff_coeff * (kl > cutoff) (kl - cutoff)^2
  float kl_coeff;        // EPI_PPOGRAD: the full d pensurr / d kl (host-computed); EPI_PPOSGD: kl_coeff
  float kl_cutoff, cutoff_coeff;
  int reverse_kl;        // kl[new, old] instead of kl[old, new]
  float* cache;          // primal activation cache (fused path) or nullptr
  int cache_mode;        // MRL_CACHE_WRITE: the forward stores h1/h2; MRL_CACHE_READ: FVP reads them
  float* feat;           // EPI_PROB with ep_t: the input rows [obs, t / limit] written beside the values
};

// [obs, t / timestep_limit] of one row (the VF fit's materialised features, core.py:659-660)
// written by the value prediction that reads them anyway: lane half h writes columns
// h, h + 2, ... of the row both halves of a 32-row tile hold
template <class XL>
__device__ __forceinline__ void write_feature_row(const RowsArgs& a, int64_t row, int h, const XL& xl) {
  const int w = a.n_obs + 1;
  float* f = a.feat + row * w;
  for (int k = h; k < w; k += 2) f[k] = xl(k);
}

constexpr float LOG2PI_F = 1.8378770664093453f;
constexpr float LOG2PIE_F = 2.8378770664093453f;

// Probtype math of one row, fp32 (the reference's floatX): the fused / layered row
// epilogues below and mrl_probtype_rows (the per-row loglik / kl / entropy the
// reference's validate_probtype checks, core.py:457-483) share these.
// Categorical on probability rows: loglik core.py:349-353, kl 355-356, entropy 358-359
__device__ __forceinline__ float cat_kl_term(float p0, float p1) { return p0 * logf(p0 / p1); }
__device__ __forceinline__ float cat_ent_term(float p) { return -(p * logf(p)); }
// DiagGauss on (mean, std[, log std]): loglik core.py:412-416, kl 421-426, entropy 428-430
__device__ __forceinline__ float gauss_kl_term(float m0, float s0, float m1, float s1) {
  const float dm = m0 - m1;
  return logf(s1 / s0) + (s0 * s0 + dm * dm) / (2.f * s1 * s1);
}
// -0.5 sum u^2 - 0.5 d log 2pi - sum log std, from sum u^2 and sum log std
__device__ __forceinline__ float gauss_loglik(float q, float sumlog, int A) {
  return -0.5f * q - 0.5f * LOG2PI_F * A - sumlog;
}
__device__ __forceinline__ float gauss_entropy(float sumlog, int A) { return sumlog + 0.5f * LOG2PIE_F * A; }

// The Fisher product's head-gradient row: the GGN metric of the KL at the old policy
// applied to the head tangent dz (== Theano's double backprop, trpo.py:45-58); g: the
// head-output part, gl: DiagGauss's log-std part (the same for every row).  Shared by the
// FVP row epilogue and the fused split Fisher product (mlp_split.hip), so both form
// these values with the same operations.
template <int MA>
__device__ __forceinline__ void fvp_metric_row(const RowsArgs& a, const float (&z)[MA], const float (&dz)[MA],
                                               const float (&sd)[MA], const float (&dls)[MA], float (&g)[MA],
                                               float (&gl)[MA]) {
  const int A = a.A;
  const float s = (float)a.inv_ng;
  for (int j = 0; j < MA; ++j) g[j] = gl[j] = 0.f;
  if (a.head == MRL_HEAD_SOFTMAX) {
    float m = z[0];
    for (int j = 1; j < A; ++j) m = fmaxf(m, z[j]);
    float p[MA], se = 0.f, pd = 0.f;
    for (int j = 0; j < A; ++j) { p[j] = expf(z[j] - m); se += p[j]; }
    for (int j = 0; j < A; ++j) { p[j] = p[j] / se; pd += p[j] * dz[j]; }
    for (int j = 0; j < A; ++j) g[j] = p[j] * (dz[j] - pd) * s;
  } else if (a.head == MRL_HEAD_GAUSS) {
    for (int j = 0; j < A; ++j) {
      g[j] = dz[j] / (sd[j] * sd[j]) * s;
      gl[j] = 2.f * dls[j] * s;
    }
  } else {
    g[0] = dz[0] * s;
  }
}

// a head-gradient store.  LDS destinations (the one-pass policy gradient's mailbox,
// mlp_fisher_hyb_kernel PROD 1) take the value through an identity DPP move first: an LDS
// op must not read a packed-f32 VALU result within 8 wait states (mlp_device.h; hipcc
// pads packed-f32 -> VALU / DPP dependencies but not -> LDS ones), and the categorical
// head's w * (onehot - p) pairs are SLP-vectorised into v_pk_mul_f32.
template <bool LDSHEAD>
__device__ __forceinline__ void st_head(float* p, float v) {
  if constexpr (LDSHEAD) v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xE4, 0xF, 0xF, false));
  *p = v;
}

template <int EPI, int MA, bool LDSHEAD = false>
__device__ __forceinline__ void row_epilogue(const RowsArgs& a, int64_t row, const float (&z)[MA],
                                             const float (&dz)[MA], const float (&ls)[MA], const float (&sd)[MA],
                                             const float (&dls)[MA], double& acc0, double& acc1, double& acc2) {
  const int A = a.A;
  if (EPI == MRL_EPI_PROB) {
    if (a.head == MRL_HEAD_LINEAR) {
      a.out[row] = z[0];
    } else if (a.head == MRL_HEAD_SOFTMAX) {
      float m = z[0];
      for (int j = 1; j < A; ++j) m = fmaxf(m, z[j]);
      float e[MA], s = 0.f;
      for (int j = 0; j < A; ++j) { e[j] = expf(z[j] - m); s += e[j]; }
      for (int j = 0; j < A; ++j) a.out[row * A + j] = e[j] / s;
    } else {
      for (int j = 0; j < A; ++j) {
        a.out[row * 2 * A + j] = z[j];
        a.out[row * 2 * A + A + j] = sd[j];
      }
    }
  } else if (EPI == MRL_EPI_LOSSES || EPI == MRL_EPI_SURRGRAD || EPI == MRL_EPI_PPOGRAD) {
    // surrogate term ratio*adv, KL and entropy of the row; SURRGRAD / PPOGRAD also write
    // the head gradient of surr (+ kl_coeff * kl for PPO)
    const float advr = a.adv[row];
    const float c = a.kl_coeff * (float)a.inv_ng;
    if (a.head == MRL_HEAD_SOFTMAX) {
      // Categorical: loglik core.py:349-353, kl 355-356, entropy 358-359
      float m = z[0];
      for (int j = 1; j < A; ++j) m = fmaxf(m, z[j]);
      float p[MA], s = 0.f;
      for (int j = 0; j < A; ++j) { p[j] = expf(z[j] - m); s += p[j]; }
      for (int j = 0; j < A; ++j) p[j] = p[j] / s;
      const int act = reinterpret_cast<const int32_t*>(a.act)[row];
      const float* op = a.oldprob + row * A;
      float pa = 0.f, opa = 0.f, kl = 0.f, ent = 0.f;
      for (int j = 0; j < A; ++j) {
        if (j == act) { pa = p[j]; opa = op[j]; }
        kl += a.reverse_kl ? cat_kl_term(p[j], op[j]) : cat_kl_term(op[j], p[j]);
        ent += cat_ent_term(p[j]);
      }
      const float ratio = expf(logf(pa) - logf(opa));
      acc0 += (double)(ratio * advr);
      acc1 += (double)kl;
      acc2 += (double)ent;
      if (EPI == MRL_EPI_SURRGRAD || EPI == MRL_EPI_PPOGRAD) {
        const float w = (float)(-a.inv_ng) * ratio * advr;
        for (int j = 0; j < A; ++j) {
          float gj = w * ((j == act ? 1.f : 0.f) - p[j]);
          if (EPI == MRL_EPI_PPOGRAD)
            gj += c * (a.reverse_kl ? p[j] * (logf(p[j] / op[j]) - kl) : p[j] - op[j]);
          st_head<LDSHEAD>(a.ghead + row * a.gh + j, gj);
        }
      }
    } else {
      // DiagGauss: loglik core.py:412-416, kl 421-426, entropy 428-430
      const float* ac = reinterpret_cast<const float*>(a.act) + row * A;
      const float* op = a.oldprob + row * 2 * A;
      float q = 0.f, q0 = 0.f, sls = 0.f, sls0 = 0.f, kl = 0.f, u[MA];
      for (int j = 0; j < A; ++j) {
        const float m0 = op[j], s0 = op[A + j];
        u[j] = (ac[j] - z[j]) / sd[j];
        const float u0 = (ac[j] - m0) / s0;
        q += u[j] * u[j];
        q0 += u0 * u0;
        sls += ls[j];
        sls0 += logf(s0);
        kl += a.reverse_kl ? gauss_kl_term(z[j], sd[j], m0, s0) : gauss_kl_term(m0, s0, z[j], sd[j]);
      }
      kl -= 0.5f * A;
      const float logp = gauss_loglik(q, sls, A);
      const float oldlogp = gauss_loglik(q0, sls0, A);
      const float ratio = expf(logp - oldlogp);
      acc0 += (double)(ratio * advr);
      acc1 += (double)kl;
      acc2 += (double)gauss_entropy(sls, A);
      if (EPI == MRL_EPI_SURRGRAD || EPI == MRL_EPI_PPOGRAD) {
        const float w = (float)(-a.inv_ng) * ratio * advr;
        for (int j = 0; j < A; ++j) {
          float gm = w * u[j] / sd[j];
          float gs = w * (u[j] * u[j] - 1.f);
          if (EPI == MRL_EPI_PPOGRAD) {
            const float m0 = op[j], s0 = op[A + j], dm = z[j] - m0;
            if (a.reverse_kl) {
              gm += c * dm / (s0 * s0);
              gs += c * (sd[j] * sd[j] / (s0 * s0) - 1.f);
            } else {
              gm += c * dm / (sd[j] * sd[j]);
              gs += c * (1.f - (s0 * s0 + dm * dm) / (sd[j] * sd[j]));
            }
          }
          st_head<LDSHEAD>(a.ghead + row * a.gh + j, gm);
          st_head<LDSHEAD>(a.ghead + row * a.gh + A + j, gs);
        }
      }
    }
  } else if (EPI == MRL_EPI_VFLOSS) {
    const float err = z[0] - a.target[row];
    acc0 += (double)err * (double)err;
    st_head<LDSHEAD>(a.ghead + row, (float)(2.0 * a.inv_ng) * err);
  } else if (EPI == MRL_EPI_FVP) {
    float g[MA], gl[MA];
    fvp_metric_row<MA>(a, z, dz, sd, dls, g, gl);
    if (a.head == MRL_HEAD_GAUSS) {
      for (int j = 0; j < A; ++j) {
        st_head<LDSHEAD>(a.ghead + row * a.gh + j, g[j]);
        st_head<LDSHEAD>(a.ghead + row * a.gh + A + j, gl[j]);
      }
    } else {
      for (int j = 0; j < A; ++j) st_head<LDSHEAD>(a.ghead + row * a.gh + j, g[j]);
    }
  }
}

}  // namespace mrl
