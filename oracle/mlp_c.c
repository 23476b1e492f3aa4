/* C restatement of the TRPO graph's batch means -- TEST INFRASTRUCTURE (oracle).
 *
 * The float64 numpy oracle (oracle/trpo_np.py) evaluates the policy gradient, the
 * Fisher-vector product and the loss means row-vectorised; at the benchmark's 4.19 M
 * Hopper rows one Fisher product there takes tens of seconds.  This file restates the
 * same per-row math in plain C (float64, one row at a time, OpenMP over contiguous row
 * blocks) so that tests can hold the device update to the float64 truth at full size:
 *
 *   mrlo_pg      d surr / d theta             trpo.py:42-43 (trpo_np.policy_gradient)
 *   mrlo_fvp     J^T M J v / N (+ 2 dlogstd)  trpo.py:45-58 (trpo_np.fisher_vector_product)
 *   mrlo_losses  [surr, kl, ent] means        trpo.py:42, 60-64 (trpo_np.surr_kl_ent)
 *
 * Network: tanh MLP, hid[0..nh-1], linear head (agentzoo.py:25-49), flat theta in Keras
 * order [W0 (in, out) row-major, b0, ..., WL, bL, (logstd)] (core.py:518-557); heads
 * 0 = DiagGauss (core.py:412-430), 1 = Categorical on softmax probabilities
 * (core.py:349-359).  Each thread sums its rows in order; the threads' partials are then
 * added in thread order, so a result depends on the thread count only through float64
 * summation order.  FMA contraction is off (the numpy oracle forms no fmas).
 * Pinned against oracle/trpo_np.py by tests/test_oracle_c.py. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXL 5
#define MAXW 1024

typedef struct {
  int n_in, nh, hid[MAXL - 1], A, head; /* head: 0 gauss, 1 softmax */
  int P;
  int64_t offW[MAXL], offb[MAXL], offls;
  int width[MAXL + 1]; /* layer input widths: width[0] = n_in, ..., width[nh + 1] = A */
} Spec;

static void spec_init(Spec* s, int n_in, int nh, const int* hid, int A, int head) {
  s->n_in = n_in;
  s->nh = nh;
  s->A = A;
  s->head = head;
  s->width[0] = n_in;
  for (int l = 0; l < nh; ++l) s->width[l + 1] = s->hid[l] = hid[l];
  s->width[nh + 1] = A;
  int64_t o = 0;
  for (int l = 0; l <= nh; ++l) {
    s->offW[l] = o;
    o += (int64_t)s->width[l] * s->width[l + 1];
    s->offb[l] = o;
    o += s->width[l + 1];
  }
  s->offls = o;
  if (head == 0) o += A;
  s->P = (int)o;
}

/* forward of one row: acts[l] = layer-l input (acts[0] = x), z = head pre-activation */
static void forward_row(const Spec* s, const double* th, const double* x, double acts[MAXL][MAXW], double* z) {
  memcpy(acts[0], x, sizeof(double) * s->n_in);
  for (int l = 0; l <= s->nh; ++l) {
    const int ni = s->width[l], no = s->width[l + 1];
    const double* W = th + s->offW[l];
    const double* b = th + s->offb[l];
    double* out = l < s->nh ? acts[l + 1] : z;
    double a[MAXW];
    for (int j = 0; j < no; ++j) a[j] = 0.0;
    for (int i = 0; i < ni; ++i) {  /* j innermost: contiguous rows of W, vectorised */
      const double xi = acts[l][i];
      const double* Wi = W + (int64_t)i * no;
      for (int j = 0; j < no; ++j) a[j] += xi * Wi[j];
    }
    for (int j = 0; j < no; ++j) out[j] = l < s->nh ? tanh(a[j] + b[j]) : a[j] + b[j];
  }
}

/* gradient accumulation of one row: g += J^T gz (no logstd slot) */
static void vjp_row(const Spec* s, const double* th, double acts[MAXL][MAXW], const double* gz, double* g) {
  double cur[MAXW], nxt[MAXW];
  memcpy(cur, gz, sizeof(double) * s->A);
  for (int l = s->nh; l >= 0; --l) {
    const int ni = s->width[l], no = s->width[l + 1];
    const double* W = th + s->offW[l];
    double* gW = g + s->offW[l];
    double* gb = g + s->offb[l];
    for (int i = 0; i < ni; ++i) {
      const double a = acts[l][i];
      for (int j = 0; j < no; ++j) gW[(int64_t)i * no + j] += a * cur[j];
    }
    for (int j = 0; j < no; ++j) gb[j] += cur[j];
    if (l > 0) {
      for (int i = 0; i < ni; ++i) {
        double t = 0.0;
        const double* Wi = W + (int64_t)i * no;
#pragma omp simd reduction(+ : t)
        for (int j = 0; j < no; ++j) t += cur[j] * Wi[j];
        nxt[i] = t * (1.0 - acts[l][i] * acts[l][i]);
      }
      memcpy(cur, nxt, sizeof(double) * ni);
    }
  }
}

/* forward-mode derivative of z along dth (trpo_np.mlp_jvp) */
static void jvp_row(const Spec* s, const double* th, const double* dth, double acts[MAXL][MAXW], double* dz) {
  double dh[MAXW], da[MAXW];
  for (int i = 0; i < s->n_in; ++i) dh[i] = 0.0;
  for (int l = 0; l <= s->nh; ++l) {
    const int ni = s->width[l], no = s->width[l + 1];
    const double* W = th + s->offW[l];
    const double* dW = dth + s->offW[l];
    const double* db = dth + s->offb[l];
    double a[MAXW], c[MAXW];
    for (int j = 0; j < no; ++j) a[j] = c[j] = 0.0;
    for (int i = 0; i < ni; ++i) {
      const double di = dh[i], xi = acts[l][i];
      const double *Wi = W + (int64_t)i * no, *dWi = dW + (int64_t)i * no;
      for (int j = 0; j < no; ++j) {
        a[j] += di * Wi[j];
        c[j] += xi * dWi[j];
      }
    }
    for (int j = 0; j < no; ++j) da[j] = a[j] + c[j] + db[j];
    if (l < s->nh) {
      for (int j = 0; j < no; ++j) dh[j] = (1.0 - acts[l + 1][j] * acts[l + 1][j]) * da[j];
    } else {
      memcpy(dz, da, sizeof(double) * no);
    }
  }
}

static void softmax_row(const double* z, int A, double* p) {
  double m = z[0], se = 0.0;
  for (int j = 1; j < A; ++j) m = z[j] > m ? z[j] : m;
  for (int j = 0; j < A; ++j) {
    p[j] = exp(z[j] - m);
    se += p[j];
  }
  for (int j = 0; j < A; ++j) p[j] /= se;
}

static const double LOG2PI = 1.8378770664093454836;

static double gauss_loglik(const double* a, const double* m, const double* sd, int d) {
  double q = 0.0, ls = 0.0;
  for (int j = 0; j < d; ++j) {
    const double u = (a[j] - m[j]) / sd[j];
    q += u * u;
    ls += log(sd[j]);
  }
  return -0.5 * q - 0.5 * LOG2PI * d - ls;
}

enum { OP_PG = 0, OP_FVP = 1, OP_LOSSES = 2 };

/* one row's contribution, unscaled by 1/N: pg / fvp add to g[P], losses to g[0..2] */
static void row_op(int op, const Spec* s, const double* th, const double* v, const double* x, const double* act,
                   double adv, const double* oldprob, double acts[MAXL][MAXW], double* g, double* crow, int fill) {
  const int A = s->A;
  double z[MAXW], gz[MAXW];
  if (crow != NULL && !fill) {  /* the primal of this theta, cached by an earlier call */
    int o = 0;
    for (int l = 0; l <= s->nh; ++l) {
      memcpy(acts[l], crow + o, sizeof(double) * s->width[l]);
      o += s->width[l];
    }
    memcpy(z, crow + o, sizeof(double) * A);
  } else {
    forward_row(s, th, x, acts, z);
    if (crow != NULL) {
      int o = 0;
      for (int l = 0; l <= s->nh; ++l) {
        memcpy(crow + o, acts[l], sizeof(double) * s->width[l]);
        o += s->width[l];
      }
      memcpy(crow + o, z, sizeof(double) * A);
    }
  }
  if (s->head == 0) {
    const double* ls = th + s->offls;
    double sd[MAXW];
    for (int j = 0; j < A; ++j) sd[j] = exp(ls[j]);
    if (op == OP_FVP) {
      double dz[MAXW];
      jvp_row(s, th, v, acts, dz);
      for (int j = 0; j < A; ++j) gz[j] = dz[j] / exp(2.0 * ls[j]);
      vjp_row(s, th, acts, gz, g);
      return;
    }
    const double logp = gauss_loglik(act, z, sd, A);
    const double oldlogp = gauss_loglik(act, oldprob, oldprob + A, A);
    const double ratio = exp(logp - oldlogp);
    if (op == OP_PG) {
      const double w = -ratio * adv;
      double* gls = g + s->offls;
      for (int j = 0; j < A; ++j) {
        const double u = (act[j] - z[j]) / sd[j];
        gz[j] = w * u / sd[j];
        gls[j] += w * (u * u - 1.0);
      }
      vjp_row(s, th, acts, gz, g);
      return;
    }
    /* losses: surr, kl(old, new), entropy */
    double kl = 0.0, ent = 0.0;
    for (int j = 0; j < A; ++j) {
      const double m0 = oldprob[j], s0 = oldprob[A + j];
      kl += log(sd[j] / s0) + (s0 * s0 + (m0 - z[j]) * (m0 - z[j])) / (2.0 * sd[j] * sd[j]);
      ent += log(sd[j]);
    }
    g[0] += -ratio * adv;
    g[1] += kl - 0.5 * A;
    g[2] += ent + 0.5 * log(2.0 * M_PI * M_E) * A;
    return;
  }
  double p[MAXW];
  softmax_row(z, A, p);
  if (op == OP_FVP) {
    double dz[MAXW], pd = 0.0;
    jvp_row(s, th, v, acts, dz);
    for (int j = 0; j < A; ++j) pd += p[j] * dz[j];
    for (int j = 0; j < A; ++j) gz[j] = p[j] * (dz[j] - pd);
    vjp_row(s, th, acts, gz, g);
    return;
  }
  const int a = (int)act[0];
  const double ratio = exp(log(p[a]) - log(oldprob[a]));
  if (op == OP_PG) {
    const double w = -ratio * adv;
    for (int j = 0; j < A; ++j) gz[j] = w * ((j == a ? 1.0 : 0.0) - p[j]);
    vjp_row(s, th, acts, gz, g);
    return;
  }
  double kl = 0.0, ent = 0.0;
  for (int j = 0; j < A; ++j) {
    kl += oldprob[j] * log(oldprob[j] / p[j]);
    ent -= p[j] * log(p[j]);
  }
  g[0] += -ratio * adv;
  g[1] += kl;
  g[2] += ent;
}

/* out[n_out] = (1/N) sum over rows of row_op, plus the row-independent logstd term of
 * the DiagGauss Fisher product (2 dlogstd). act: [N, A] (gauss) or [N] as doubles. */
static int run(int op, int n_in, int nh, const int* hid, int A, int head, const double* th, const double* v,
               const double* ob, const double* act, const double* adv, const double* oldprob, int64_t N, int threads,
               double* out, double* cache, int fill) {
  if (nh < 0 || nh > MAXL - 1 || A < 1 || A > MAXW || n_in < 1 || n_in > MAXW || N < 1) return -1;
  for (int l = 0; l < nh; ++l)
    if (hid[l] < 1 || hid[l] > MAXW) return -1;
  Spec s;
  spec_init(&s, n_in, nh, hid, A, head);
  const int n_out = op == OP_LOSSES ? 3 : s.P;
  const int T = threads > 0 ? threads : 1;
  double* part = (double*)calloc((size_t)T * n_out, sizeof(double));
  if (!part) return -2;
  const int pw = head == 0 ? 2 * A : A;  /* oldprob row width */
  const int aw = head == 0 ? A : 1;      /* action row width */
  int cw = A;                             /* cached row: every layer's input, then z */
  for (int l = 0; l <= nh; ++l) cw += s.width[l];
#pragma omp parallel num_threads(T)
  {
#ifdef _OPENMP
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
#else
    const int t = 0, nt = 1;
#endif
    double(*acts)[MAXW] = (double(*)[MAXW])malloc(sizeof(double) * MAXL * MAXW);
    double* g = part + (size_t)t * n_out;
    const int64_t lo = N * t / nt, hi = N * (t + 1) / nt;
    for (int64_t r = lo; r < hi; ++r)
      row_op(op, &s, th, v, ob + r * n_in, act ? act + r * aw : NULL, adv ? adv[r] : 0.0,
             oldprob ? oldprob + r * pw : NULL, acts, g, cache ? cache + r * cw : NULL, fill);
    free(acts);
  }
  for (int k = 0; k < n_out; ++k) {
    double a = 0.0;
    for (int t = 0; t < T; ++t) a += part[(size_t)t * n_out + k];
    out[k] = a / (double)N;
  }
  if (op == OP_FVP && head == 0)
    for (int j = 0; j < A; ++j) out[s.offls + j] = 2.0 * v[s.offls + j];
  free(part);
  return 0;
}

int mrlo_n_params(int n_in, int nh, const int* hid, int A, int head) {
  Spec s;
  if (nh < 0 || nh > MAXL - 1) return -1;
  spec_init(&s, n_in, nh, hid, A, head);
  return s.P;
}

/* cache (optional): [N, n_in + sum(hid) + A] doubles, the primal of theta; fill = 1 writes
 * it, fill = 0 reads it instead of the forward (the caller keys it to theta) */
int mrlo_pg(int n_in, int nh, const int* hid, int A, int head, const double* th, const double* ob, const double* act,
            const double* adv, const double* oldprob, int64_t N, int threads, double* g, double* cache, int fill) {
  return run(OP_PG, n_in, nh, hid, A, head, th, NULL, ob, act, adv, oldprob, N, threads, g, cache, fill);
}

int mrlo_fvp(int n_in, int nh, const int* hid, int A, int head, const double* th, const double* v, const double* ob,
             int64_t N, int threads, double* fv, double* cache, int fill) {
  return run(OP_FVP, n_in, nh, hid, A, head, th, v, ob, NULL, NULL, NULL, N, threads, fv, cache, fill);
}

int mrlo_losses(int n_in, int nh, const int* hid, int A, int head, const double* th, const double* ob,
                const double* act, const double* adv, const double* oldprob, int64_t N, int threads, double* out3,
                double* cache, int fill) {
  return run(OP_LOSSES, n_in, nh, hid, A, head, th, NULL, ob, act, adv, oldprob, N, threads, out3, cache, fill);
}
