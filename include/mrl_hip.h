/* libmrl_hip -- C ABI of the MI355X-native TRPO hot path (gfx950 HIP kernels).
 *
 * The reference (ddlau/modular_rl) has no native code and no FFI: its hot path is
 * Theano-compiled graphs and numpy called from Python.  This
 * header is the boundary the Python host layer (`modular_rl_amd/_lib.py`, ctypes)
 * binds; each entry cites the reference interface it replaces.
 *
 * Conventions
 *  - Every function returns 0 on success, <0 on error (MRL_E_*); the message is in
 *    mrl_last_error().  No C++ exception crosses the ABI.
 *  - All buffers are caller-owned DEVICE pointers (e.g. torch.Tensor.data_ptr());
 *    every call is asynchronous on `stream` (a hipStream_t), no host sync, no
 *    allocation -- so the whole hot path can be captured in a hipGraph.
 *  - Row n of every [N, ...] batch array is time-major: n = t * n_envs + e.
 *  - `skip` (may be NULL): device int; when *skip != 0 the kernel returns at once
 *    (device-side early exit of the conjugate-gradient loop, trpo.py:192-193).
 */
#ifndef MRL_HIP_H
#define MRL_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRL_OK 0
#define MRL_E_ARG (-1)
#define MRL_E_UNSUPPORTED (-2)
#define MRL_E_HIP (-3)

/* head kinds */
#define MRL_HEAD_LINEAR 0   /* value net, Dense(1)                 agentzoo.py:58      */
#define MRL_HEAD_SOFTMAX 1  /* Categorical, Dense(k, softmax)      agentzoo.py:46      */
#define MRL_HEAD_GAUSS 2    /* DiagGauss, Dense(d) + ConcatFixedStd agentzoo.py:40-43 */

/* tanh MLP shape: n_in -> 64 -> 64 -> n_out (the fast path; hid_sizes=[64,64],
 * agentzoo.py:20-23).  Other shapes return MRL_E_UNSUPPORTED (no CPU fallback). */
typedef struct {
  int32_t n_in;    /* input features (obs dim, +1 for the VF time feature)   */
  int32_t n_out;   /* k (Categorical), d (DiagGauss) or 1 (value)             */
  int32_t head;    /* MRL_HEAD_*                                              */
  int32_t n_hidden;/* must be 64                                              */
  int32_t n_layers;/* must be 2                                               */
  int32_t cus;     /* CUs the VJP and the row passes with partial sums are
                    * sized for (0: all 256; other row passes use the device):
                    * the grid caps scale with it, so passes issued on a stream
                    * restricted to that many CUs run in whole rounds.  Part of
                    * the result's identity: the per-wave partial sums follow
                    * the grid, so runs compared bit for bit use the same value */
} mrl_mlp_desc;

const char* mrl_last_error(void);
int32_t mrl_version(void);

/* number of float parameters (flat theta, Keras trainable_weights order,
 * core.py:518-557) and of floats in the packed LDS image */
int64_t mrl_mlp_num_params(const mrl_mlp_desc* d);
int64_t mrl_mlp_image_floats(const mrl_mlp_desc* d);

/* theta (fp32 flat) -> image.  Replaces SetFromFlat (core.py:527-541): the
 * kernels read weights only through the image.  fwd_only: skip backward frags. */
int mrl_mlp_pack(const mrl_mlp_desc* d, const float* theta, float* image, int32_t fwd_only,
                 const int32_t* skip, void* stream);

/* row epilogues of the fused forward pass (mrl_mlp_rows) */
#define MRL_EPI_PROB 0      /* out <- prob rows [N,k] / [N,2d] / value [N]     core.py:261-270, 648-650 */
#define MRL_EPI_LOSSES 1    /* partial <- (sum ratio*adv, sum KL(old,new), sum ent)  trpo.py:60-64    */
#define MRL_EPI_SURRGRAD 2  /* LOSSES + ghead <- d surr / d head rows              trpo.py:42-43     */
#define MRL_EPI_VFLOSS 3    /* partial <- sum (y-yhat)^2; ghead <- 2(yhat-y)/N_glob core.py:611-617  */
#define MRL_EPI_FVP 4       /* forward + JVP(tangent) + KL metric -> ghead rows      trpo.py:45-58   */
#define MRL_EPI_PPOGRAD 5   /* LOSSES + ghead <- d(surr + kl_coeff * kl)/d head rows; kl_coeff = the
                               whole d pensurr / d kl, host-computed            ppo.py:46-52       */
#define MRL_EPI_PPOSGD 6    /* one launch = one minibatch of n <= MRL_PPO_BLOCK_ROWS rows: block-reduced
                               kl, c = kl_coeff + 2 cutoff_coeff (kl - cutoff)+, ghead of pensurr
                               (ppo.py:150-156); partial sums as LOSSES                            */
#define MRL_PPO_BLOCK_ROWS 128

typedef struct {
  const float* x;          /* [N, n_obs] observations                              */
  const int32_t* ep_t;     /* [N] step index in episode (VF time feature) or NULL  */
  double timestep_limit;   /* time feature = ep_t / timestep_limit (core.py:660)   */
  int64_t n;               /* rows                                                 */
  double inv_n_global;     /* 1 / rows summed over all ranks                       */
  const void* act;         /* [N] int32 (Categorical) | [N, d] float (DiagGauss)   */
  const float* adv;        /* [N] standardized advantages                          */
  const float* oldprob;    /* [N, k] | [N, 2d] rollout-time prob rows              */
  const float* target;     /* [N] VF regression target                             */
  float* out;              /* EPI_PROB output                                      */
  float* ghead;            /* [N, gh] head-gradient rows (gh = k, 2d or 1)         */
  double* partial;         /* [mrl_partial_rows(n), 4] fp64 per-wave partial sums  */
  double kl_coeff;         /* PPO epilogues (see MRL_EPI_PPOGRAD / PPOSGD)         */
  double kl_cutoff;        /* PPOSGD: 2 * kl_target                                */
  double cutoff_coeff;     /* PPOSGD: kl_cutoff_coeff (1000)                       */
  int32_t reverse_kl;      /* kl[new, old] instead of kl[old, new] (PpoLbfgs)     */
  int32_t cache_mode;      /* MRL_CACHE_* (fused path; act_cache NULL = no cache) */
  float* act_cache;        /* [mrl_act_cache_floats(n)] primal h1/h2 of theta     */
  float* feat_out;         /* MRL_EPI_PROB with ep_t only, else NULL: the rows the
                            * pass reads, [N, n_obs + 1] = [x, ep_t / timestep_limit]
                            * (NnVf.preproc, core.py:659-660), written beside the
                            * values for the VF fit -- bitwise mrl_concat_time's X   */
} mrl_rows_io;

/* Primal activation cache of the fused path: the forward of one theta is shared by
 * every Fisher product of an update (trpo.py:70 is called 10-11 times at a fixed
 * theta) and by the VJP that follows a loss pass.  A plain-forward epilogue (PROB,
 * LOSSES, SURRGRAD, VFLOSS, PPOGRAD) with MRL_CACHE_WRITE stores h1/h2; EPI_FVP with
 * MRL_CACHE_READ and mrl_mlp_vjp with a non-NULL cache read them instead of
 * recomputing the forward (bitwise the same activations). */
#define MRL_CACHE_NONE 0
#define MRL_CACHE_WRITE 1
#define MRL_CACHE_READ 2
int64_t mrl_act_cache_floats(int64_t n);

int64_t mrl_partial_rows(int64_t n);  /* rows of `partial` a call over n rows writes */
int64_t mrl_slab_rows(int64_t n);     /* rows of the mrl_mlp_vjp slab                */
/* the same for a desc whose `cus` is set (the two above: cus = 0) */
int64_t mrl_mlp_partial_rows(const mrl_mlp_desc* d, int64_t n);
int64_t mrl_mlp_slab_rows(const mrl_mlp_desc* d, int64_t n);

/* fused forward (+ JVP for EPI_FVP) with a per-row epilogue.
 * theta: flat fp32 params (for logstd); image: packed primal image;
 * tangent/image_t: flat fp32 tangent and its packed image (EPI_FVP only). */
int mrl_mlp_rows(const mrl_mlp_desc* d, int32_t epilogue, const float* theta, const float* image,
                 const float* tangent, const float* image_t, const mrl_rows_io* io,
                 const int32_t* skip, void* stream);

/* vector-Jacobian product: slab[w, :] <- per-wave partial of sum_n J_n^T ghead_n in
 * flat theta layout (head columns beyond n_out -- DiagGauss logstd -- are summed
 * into the logstd slots).  Replaces flatgrad / the VJP half of the Theano Fvp.
 * act_cache: the primal activations of the same theta and rows (MRL_CACHE_WRITE of a
 * preceding pass), or NULL to recompute the forward. */
int mrl_mlp_vjp(const mrl_mlp_desc* d, const float* image, const float* x, const int32_t* ep_t,
                double timestep_limit, const float* ghead, int64_t n, float* slab, const float* act_cache,
                const int32_t* skip, void* stream);

/* out[c] = sum_r slab[r, c] in fixed order with fp64 accumulation */
/* bf16 throughput mode of the three fused passes above (MRL_COMPUTE_BF16,
 * csrc/mlp_bf16.hip): same arguments and semantics, bf16 MFMA operands (weights, layer
 * inputs, backpropagated rows) with f32 accumulation; f32 biases / tanh / head /
 * epilogues.  `image` is the bf16 image (mrl_mlp_pack_bf16, mrl_mlp_image_words_bf16
 * 4-byte words), `act_cache` the bf16 activation cache (mrl_act_cache_words_bf16);
 * partial / slab buffers are sized by the _bf16 row counts.  fp32 stays the parity
 * dtype (north_star 1e-4); bf16 is checked at a bf16 bound. */
int64_t mrl_mlp_image_words_bf16(const mrl_mlp_desc* d);
int64_t mrl_act_cache_words_bf16(int64_t n);
int64_t mrl_partial_rows_bf16(int64_t n);
int64_t mrl_slab_rows_bf16(int64_t n);
int64_t mrl_mlp_partial_rows_bf16(const mrl_mlp_desc* d, int64_t n);
int64_t mrl_mlp_slab_rows_bf16(const mrl_mlp_desc* d, int64_t n);
int mrl_mlp_pack_bf16(const mrl_mlp_desc* d, const float* theta, float* image, int32_t fwd_only,
                      const int32_t* skip, void* stream);
int mrl_mlp_rows_bf16(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image,
                      const float* tangent, const float* image_t, const mrl_rows_io* io, const int32_t* skip,
                      void* stream);
int mrl_mlp_vjp_bf16(const mrl_mlp_desc* d, const float* image, const float* x, const int32_t* ep_t, double ts_limit,
                     const float* ghead, int64_t n, float* slab, const float* act_cache, const int32_t* skip,
                     void* stream);

/* The fp32-accurate Fisher product's JVP half on bf16 MFMA (csrc/mlp_split.hip): every
 * f32 MFMA operand split exactly into three bf16 parts, the part products accumulated in
 * f32 (6 of the 9, the dropped three <= 2^-25 of the product: below one f32 ulp).  Same
 * semantics as mrl_mlp_rows(MRL_EPI_FVP) with MRL_CACHE_READ (the f32 activation cache of
 * a preceding f32 SURRGRAD / LOSSES pass) -- trpo.py:45-58, 70; the images are split
 * images of the forward weights (mrl_mlp_pack_split, for theta and for the tangent).  The
 * VJP half is mrl_mlp_vjp with the cache. */
int64_t mrl_mlp_image_words_split(const mrl_mlp_desc* d);
int mrl_mlp_pack_split(const mrl_mlp_desc* d, const float* theta, float* image, const int32_t* skip, void* stream);
int mrl_mlp_fvp_split(const mrl_mlp_desc* d, const float* theta, const float* image, const float* tangent,
                      const float* image_t, const mrl_rows_io* io, const int32_t* skip, void* stream);
/* The whole Fisher product in one launch (trpo.py:45-58, Fvp = J^T M J v): per block,
 * four waves run the split JVP rows above on 32-row tiles and leave the KL-metric head
 * rows in LDS, four waves run the hybrid cached VJP (mrl_mlp_vjp) on them; the activation
 * cache crosses HBM once.  Slab rows as mrl_mlp_vjp (mrl_mlp_slab_rows(d, n)), then
 * mrl_reduce_rows_f32.  image: the f32 image (its W1 / W2 fragments); image_s / image_t_s:
 * split images of theta and of the tangent.  E_UNSUPPORTED unless
 * mrl_mlp_fisher_hyb_fits(d) (policy nets of <= 15 inputs; the split images fit LDS). */
/* The forward row passes PROB / LOSSES / SURRGRAD / VFLOSS of mrl_mlp_rows (same io, same
 * grid and partial rows, MRL_CACHE_WRITE stores the same activation-cache layout) on the
 * split image of theta (mrl_mlp_pack_split): both layers as six bf16 part products, f32
 * accumulation -- the f32 kernel's per-row values to f32 rounding (core.py:261-270,
 * 611-617, 648-650; trpo.py:42-43, 60-64). */
int mrl_mlp_rows_split(const mrl_mlp_desc* d, int32_t epi, const float* theta, const float* image_s,
                       const mrl_rows_io* io, const int32_t* skip, void* stream);
int32_t mrl_mlp_fisher_hyb_fits(const mrl_mlp_desc* d);
int mrl_mlp_fisher_hyb(const mrl_mlp_desc* d, const float* theta, const float* image, const float* image_s,
                       const float* tangent, const float* image_t_s, const mrl_rows_io* io, float* slab,
                       const int32_t* skip, void* stream);
/* The policy gradient in ONE launch (trpo.py:42-43, the surrogate's flat gradient; round
 * 6): mrl_mlp_rows_split's SURRGRAD pass (io: x, n, inv_n_global, act, adv, oldprob,
 * partial; act_cache with MRL_CACHE_WRITE, written as that pass writes it) beside the
 * hybrid VJP of mrl_mlp_vjp in each block, the head-gradient rows through LDS (no ghead in
 * HBM).  slab: mrl_mlp_slab_rows(d, n) rows of P floats (reduce with mrl_reduce_rows_f32);
 * partial: the same number of rows of 4 doubles (surr, kl, ent, 0 sums; reduce with
 * mrl_reduce_rows_f64).  Same shapes as mrl_mlp_fisher_hyb (mrl_mlp_fisher_hyb_fits). */
int mrl_mlp_grad_hyb(const mrl_mlp_desc* d, const float* theta, const float* image, const float* image_s,
                     const mrl_rows_io* io, float* slab, const int32_t* skip, void* stream);

int mrl_reduce_rows_f32(const float* slab, int64_t rows, int64_t cols, float* out, const int32_t* skip, void* stream);
int mrl_reduce_rows_f64(const double* slab, int64_t rows, int64_t cols, double* out, const int32_t* skip, void* stream);

/* ---------------------------------------------------------------- layered (wide) MLP path
 * Any hid_sizes (e.g. Humanoid 376-512-512-512-17): each Dense layer
 * is one tiled fp32-MFMA GEMM over all rows (forward, JVP, input-grad, weight-grad)
 * and the head epilogue is a per-row kernel; the host sequences them
 * (modular_rl_amd/nets.py LayeredMlpNet).  Replaces the same Theano functions as
 * mrl_mlp_rows / mrl_mlp_vjp for nets the fused 64-wide kernels do not cover. */
#define MRL_LAYERED_MAX_OUT 32

#define MRL_GEMM_STORE 0  /* C = AB (+ bias)                                         */
#define MRL_GEMM_TANH 1   /* C = tanh(AB + bias)                  Dense + tanh forward */
#define MRL_GEMM_DTANH 2  /* C = (AB + bias) * (1 - H^2)          JVP / input-grad    */
/* operand precision of the MFMA passes (fp32 is the parity dtype, north_star 1e-4;
 * bf16 is the throughput mode: operands rounded to bf16 RNE, f32 accumulation) */
#define MRL_COMPUTE_F32 0
#define MRL_COMPUTE_BF16 1
#define MRL_COMPUTE_SPLIT 2 /* fp32 on split bf16 operands (mrl_mlp_rows_split; mrl_linesearch_eval) */
#define MRL_GEMM_SLAB 3   /* c + z*slab_stride = sum over K-split z of AB  (weight grads) */

typedef struct {
  int64_t m, n, k;
  const float* a;       /* op(a)(i,k) = a[i*lda+k] (a_trans 0) | a[k*lda+i] (a_trans 1)  */
  int64_t lda;
  int32_t a_trans;
  int32_t ones_row;     /* 1: row m-1 of op(a) is all ones (bias grad rides the weight-grad GEMM) */
  const float* b;       /* op(b)(k,j) = b[k*ldb+j] (b_trans 0) | b[j*ldb+k] (b_trans 1)  */
  int64_t ldb;
  int32_t b_trans;
  int32_t epilogue;     /* MRL_GEMM_*                                                    */
  const float* a2;      /* optional second product a2.b2 (same shapes/layout) added to C  */
  const float* b2;
  float* c;
  int64_t ldc;
  const float* bias;    /* [n] or NULL                                                   */
  const float* h;       /* MRL_GEMM_DTANH: [m, ldh] activations                          */
  int64_t ldh;
  int32_t splits;       /* MRL_GEMM_SLAB: requested K splits (see mrl_gemm_slab_splits)  */
  int32_t compute;      /* MRL_COMPUTE_F32 (exact f32 MFMA) | MRL_COMPUTE_BF16 (bf16 operands, f32 accumulate) */
  int64_t slab_stride;  /* MRL_GEMM_SLAB: floats between consecutive split slabs         */
} mrl_gemm_desc;

int mrl_gemm(const mrl_gemm_desc* g, const int32_t* skip, void* stream);
/* column-tile width mrl_gemm launches for this descriptor: 32 (narrow 128x32 tiles: n <= 32
 * or fewer than 160 128x128 blocks) or 128 (0 for an empty product); host-only query */
int32_t mrl_gemm_tile_n(const mrl_gemm_desc* g);

/* bf16-operand GEMMs of the layered path's bf16 mode (csrc/gemm_bf16.hip): operands in
 * HBM as bf16 (a bf16 tape and packed bf16 weight images), f32 accumulation.  The
 * reference interface they serve is the same as mrl_gemm's (Keras Dense layers,
 * agentzoo.py:34-48, and their Theano gradients, trpo.py:40-47). */
typedef struct {
  int64_t m, n, k;
  const uint16_t* a;    /* bf16 [m, lda] row-major, k contiguous; columns k..lda-1 zero   */
  int64_t lda;          /* multiple of 8                                                  */
  const uint16_t* bt;   /* B transposed: bf16 [n, ldb] (k contiguous), zero padding       */
  int64_t ldb;          /* multiple of 8                                                  */
  const uint16_t* a2;   /* optional second product a2 . bt2^T (same k / lda / ldb)         */
  const uint16_t* bt2;
  void* c;              /* [m, ldc] f32, or bf16 when c_bf16                              */
  int64_t ldc;
  int32_t c_bf16;
  int32_t epilogue;     /* MRL_GEMM_STORE | MRL_GEMM_TANH | MRL_GEMM_DTANH                */
  const float* bias;    /* [n] or NULL                                                    */
  const uint16_t* h;    /* DTANH: bf16 [m, ldh] activations                               */
  int64_t ldh;
  int32_t lds_limit;    /* 0, or the LDS bytes per block the GEMM may use: only kernels of
                         * at most that footprint, never the persistent CU-holding ones (a
                         * GEMM co-scheduled beside the wave-per-env rollout); same results */
} mrl_gemm_bf16_desc;
int mrl_gemm_bf16(const mrl_gemm_bf16_desc* g, const int32_t* skip, void* stream);

/* weight gradients: slab[z*slab_stride + i*ldc + j] = sum over row split z of
 * a[r, i] * b[r, j] (both bf16 row-major over the k rows); ones_row: row m-1 of the
 * result is the column sums of b (the bias gradient: a's column m-1 reads as 1).
 * Splits as mrl_gemm_slab_splits(k, splits). */
typedef struct {
  int64_t m, n, k;
  const uint16_t* a;
  int64_t lda;
  const uint16_t* b;
  int64_t ldb;
  int32_t ones_row;
  int32_t splits;
  float* slab;
  int64_t slab_stride, ldc;
  int32_t lds_limit;    /* as mrl_gemm_bf16_desc.lds_limit */
} mrl_gemm_bf16_tn_desc;
int mrl_gemm_bf16_tn(const mrl_gemm_bf16_tn_desc* g, const int32_t* skip, void* stream);
/* y[r, c] = bf16(x[r, c]) (RNE) for c < cols, 0 for cols <= c < ldy */
int mrl_cast_rows_bf16(const float* x, int64_t rows, int64_t cols, int64_t ldx, uint16_t* y, int64_t ldy,
                       void* stream);
/* bf16 image of a Dense kernel W [din, dout] (f32): transpose 0 -> [din, ld] = W,
 * transpose 1 -> [dout, ld] = W^T; zero padding columns */
int mrl_pack_w_bf16(const float* w, int64_t din, int64_t dout, int32_t transpose, uint16_t* out, int64_t ld,
                    void* stream);
/* slabs a MRL_GEMM_SLAB call over k rows with `max_splits` requested actually writes */
int64_t mrl_gemm_slab_splits(int64_t k, int32_t max_splits);
/* bias / logstd gradients: slab[z*slab_stride + c] = sum of g[r, c] (ld ldg) over the
 * z-th of `splits` equal row chunks, z < splits (empty chunks write 0) */
int mrl_colsum(const float* g, int64_t m, int64_t n, int64_t ldg, int32_t splits, float* slab, int64_t slab_stride,
               const int32_t* skip, void* stream);
/* per-row head epilogue (same semantics as mrl_mlp_rows' epilogues) on head rows
 * z [N, n_out] (and tangent rows dz for EPI_FVP); logstd/dlogstd for DiagGauss;
 * io->x / ep_t unused; partial has mrl_partial_rows(n) rows. */
int mrl_head_rows(int32_t head, int32_t n_out, int32_t epilogue, const float* z, const float* dz,
                  const float* logstd, const float* dlogstd, const mrl_rows_io* io, const int32_t* skip,
                  void* stream);
/* X[N, n_obs+1] = [obs, ep_t/timestep_limit]  (value-net input, core.py:659-660);
 * max_blocks > 0 caps the grid (a copy run beside other work), 0: the whole device */
int mrl_concat_time(const float* obs, const int32_t* ep_t, int64_t n, int32_t n_obs, double timestep_limit,
                    float* x, int32_t max_blocks, void* stream);

/* ---------------------------------------------------------------- conjugate gradient
 * Device-resident Demmel CG on flat fp64 vectors (trpo.py:165-200).
 * state (fp64): [0]=rdotr [1]=last pz [2]=iterations run; flag (int32[2]): [0]=converged.
 * init:   x=0, r=p=b, rdotr=r.r, p32=(float)p, flag=0, ax=0.
 * update: z = fvp + damping*p; v=rdotr/p.z; x+=v p; ax+=v z; r-=v z; mu=r.r/rdotr; p=r+mu p;
 *         flag=1 when rdotr<tol; pass `flag` as the `skip` of the next Fvp kernels.
 * ax (fp64 [n], optional: NULL skips it) accumulates (F + damping I) x, which the
 * step scaling needs (trpo.py:119-122) -- A is linear, so A sum v_k p_k = sum v_k z_k
 * and no Fisher product of the step direction has to be run.
 * `state` (and the `out` of mrl_trpo_step_ax) must hold mrl_cg_state_doubles(n) doubles:
 * above 65,536 elements the passes run on 256 blocks and keep their block partials
 * there (wide nets, e.g. Humanoid P = 727,074). */
int64_t mrl_cg_state_doubles(int64_t n);
int mrl_cg_init(const double* b, int64_t n, double* x, double* r, double* p, float* p32, double* ax,
                double* state, int32_t* flag, void* stream);
int mrl_cg_update(const float* fvp, double damping, double residual_tol, int64_t n, double* x, double* r,
                  double* p, float* p32, double* ax, double* state, int32_t* flag, void* stream);
/* mrl_cg_update that also writes the next Fisher product's split tangent image of p32
 * (what mrl_mlp_pack_split(d, p32, image_t) writes), so the CG loop issues one launch
 * fewer per iteration; the single-block update only (n <= 8192, else E_UNSUPPORTED),
 * n must be d's parameter count */
int mrl_cg_update_pack(const float* fvp, double damping, double residual_tol, int64_t n, double* x, double* r,
                       double* p, float* p32, double* ax, double* state, int32_t* flag, const mrl_mlp_desc* d,
                       float* image_t, void* stream);
/* step scaling (trpo.py:119-124): shs = .5 x.(fvp + damping x), lm = sqrt(shs/max_kl),
 * fullstep = x/lm, out[0]=shs out[1]=lm out[2]=-g.x out[3]=-g.x/lm (expected rate) */
int mrl_trpo_step(const float* fvp, const double* x, const float* g, double damping, double max_kl,
                  int64_t n, double* fullstep, double* out, void* stream);
/* the same scaling from ax = (F + damping I) x accumulated by mrl_cg_update:
 * shs = .5 x.ax (the update path: one Fisher product fewer per TRPO step) */
int mrl_trpo_step_ax(const double* ax, const double* x, const float* g, double max_kl, int64_t n,
                     double* fullstep, double* out, void* stream);
/* theta_out = (float)(theta_old + frac * fullstep)   (linesearch, trpo.py:150, core.py:540) */
int mrl_axpy_cast(const float* theta_old, const double* fullstep, double frac, int64_t n, float* theta_out,
                  void* stream);
/* ---------------------------------------------------------------- batched line search
 * The backtracking line search (trpo.py:143-159) scores candidates theta_k =
 * (float)(theta_old + 0.5^(k0+k) fullstep) (stepfrac k0+k; SetFromFlat's cast, core.py:540).
 * candidates: out [K, n], one launch (0 < K, k0 + K <= 64). */
int mrl_linesearch_candidates(const float* theta_old, const double* fullstep, int32_t k0, int32_t K, int64_t n,
                              float* out, void* stream);
/* Fused 64-wide policy: the K candidates scored in one call -- candidates into cand [K, P],
 * per candidate its forward image (images + k*image_stride; f32 image floats or bf16 image
 * words by `compute`, MRL_COMPUTE_*), a MRL_EPI_LOSSES pass over io's rows into partials +
 * k*partial_stride ([partial rows, 4] fp64; io->partial / act_cache ignored) and out[k*4..] =
 * (sum ratio*adv, sum kl, sum entropy, rows): the caller reads out back ONCE (one all-reduce
 * of [K, 4] in data-parallel mode) and takes the first k whose ratio passes, as the
 * reference's serial loop does.  Replaces K rounds of compute_losses + readback. */
int mrl_linesearch_eval(const mrl_mlp_desc* pol, int32_t compute, const float* theta_old, const double* fullstep,
                        int32_t k0, int32_t K, const mrl_rows_io* io, float* cand, float* images,
                        int64_t image_stride, double* partials, int64_t partial_stride, double* out, void* stream);
/* Adam in floatX (PpoSgdUpdater's adam_updates, ppo.py:231-258): m, v, theta fp32 [n];
 * a_t = lr sqrt(1-b2^t)/(1-b1^t) computed by the caller */
int mrl_adam_step(float* theta, const float* g, float* m, float* v, double a_t, double beta1, double beta2,
                  double eps, int64_t n, void* stream);
/* dst row i = src row idx[i] (row_bytes a multiple of 4): PPO minibatch permutation */
int mrl_gather_rows(const void* src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst, void* stream);
/* out (fp64) = scale * (double)in ; in-place-safe */
int mrl_cast_scale_f32_f64(const float* in, double scale, int64_t n, double* out, void* stream);

/* Per-row probtype values on probability rows (the reference's Categorical /
 * DiagGauss loglik, kl, entropy: core.py:349-359, 412-430), computed by the same fp32
 * device helpers as the MLP row epilogues.  head MRL_HEAD_SOFTMAX: prob [n, k], x
 * int32 [n]; MRL_HEAD_GAUSS: prob [n, 2k] = [mean | std], x fp32 [n, k].
 * loglik[r] = log p(x_r), kl[r] = KL(prob_r || prob2_r), ent[r] = entropy(prob_r); any
 * output may be NULL.  The reference checks them with validate_probtype (core.py:457-483). */
int mrl_probtype_rows(int32_t head, int32_t k, int64_t n, const float* prob, const float* prob2, const void* x,
                      float* loglik, float* kl, float* ent, void* stream);

/* ---------------------------------------------------------------- advantage
 * GAE + discounted return over time-major [T, E] rows (core.py:63-75 with
 * misc_utils.py:9-27 discount): flags bit0 = episode ends at this row, bit1 = the
 * env terminated (bootstrap 0) else bootstrap with the row's own baseline (core.py:73).
 * moments (fp64 [3]) <- (sum adv, sum adv^2, count)  (for core.py:100-105).
 * workspace: mrl_gae_workspace_bytes(T, E) bytes, ZEROED before its first mrl_gae and
 * not written by anything else between calls (it holds a completion counter that each
 * call returns to 0); one workspace per stream of concurrent calls. */
int mrl_gae(const float* rew, const float* vpred, const uint8_t* flags, int64_t T, int64_t E, double gamma,
            double lam, float* adv, float* ret, double* moments, void* workspace, void* stream);
int64_t mrl_gae_workspace_bytes(int64_t T, int64_t E);
/* adv <- (adv - mean)/std, numpy std (ddof=0, no eps) as its two passes (core.py:100-105):
 * moments = (sum, sumsq, n) of the first pass (mrl_gae), cmoments = (sum, sumsq, n) of
 * (adv - moments[0]/moments[2]) from mrl_moments_centered (both summed over ranks).
 * cmoments may be NULL: single-pass E[x^2]-mean^2 (cancels when |mean| >> std). */
int mrl_standardize(float* adv, int64_t n, const double* moments, const double* cmoments, void* stream);
/* y = mixfrac * ret + (1 - mixfrac) * vpred  (NnRegression.fit target, core.py:622-624) */
int mrl_vf_target(const float* ret, const float* vpred, double mixfrac, int64_t n, float* y, void* stream);
/* out (fp64 [3]) <- (sum (a-b), sum (a-b)^2, n); b may be NULL.  For the VF stats
 * (PredStdev / TargStdev / explained variance, core.py:629-636, misc_utils.py:29-49) */
int mrl_moments(const float* a, const float* b, int64_t n, double* out, void* workspace, void* stream);
/* out (fp64 [3]) <- (sum d, sum d^2, n) of d = a - b - center[0]/center[2] (center: a
 * device fp64 [3] from a previous mrl_moments / mrl_gae pass): the second pass of a
 * two-pass variance, var = out[1]/n - (out[0]/n)^2, with no cancellation */
int mrl_moments_centered(const float* a, const float* b, int64_t n, const double* center, double* out,
                         void* workspace, void* stream);
int64_t mrl_moments_workspace_bytes(int64_t n);
/* episode statistics of the batch (add_episode_stats, core.py:31-44): out (fp64 [6]) <-
 * (n_episodes, sum R, sum R^2, max R, sum len, max len); an episode = a row run ending
 * at a flags&1 row (whole episode, or a horizon-cut one, like a reference path). */
int mrl_episode_stats(const float* rew, const uint8_t* flags, int64_t T, int64_t E, double* out, void* workspace,
                      void* stream);
int64_t mrl_episode_stats_workspace_bytes(int64_t E);

/* ---------------------------------------------------------------- batched rollout
 * Replaces do_rollouts_serial/rollout (core.py:174-221) + ZFilter (filters.py:17-40)
 * + StochPolicy.act (core.py:261-267) + gym env.step: E envs step in lock-step on
 * device for T steps.  Per step the E new observations are merged into the running
 * stat (Chan merge of per-block Welford partials in block order), then normalised. */
#define MRL_ENV_CARTPOLE 0  /* CartPole-v0 equations (gym), k = 2            */
#define MRL_ENV_HOPPER 1    /* Hopper-v2: hopper.xml articulated body, obs 11 / act 3 */
#define MRL_ENV_HUMANOID 2  /* Humanoid-v2: humanoid.xml articulated body, obs 376 / act 17 (layered rollout only) */

typedef struct {
  int32_t env_id;          /* MRL_ENV_*                                          */
  int32_t n_envs;          /* E on this rank                                     */
  int32_t horizon;         /* T steps per iteration                              */
  int32_t timestep_limit;  /* episode cut (core.py:190, run_pg.py:103-105)       */
  int32_t filter;          /* 1: ZFilter obs (clip 5) + reward RunningStat       */
  int32_t env_offset;      /* rank * E: global env id for the RNG streams         */
  uint64_t seed;           /* Philox key                                         */
  int32_t compute;         /* MRL_COMPUTE_*: the policy net's dtype; BF16 rounds the
                              fused forward's W0, W1, x, h1, h2 to bf16 like
                              mrl_mlp_rows_bf16, so rollout prob rows = update's    */
  int32_t launch_cus;      /* mrl_rollout_run's residency check: 0 = the CUs of the
                              stream it is called on; > 0 = the CUs of the stream a
                              captured graph will be replayed on (capture streams
                              carry no CU mask); < 0 = debug only, skip the check
                              (a non-resident grid then aborts: sync[32] != 0)       */
} mrl_rollout_desc;

typedef struct {
  double* env_state;       /* [state_doubles, E]: SoA state rows (Humanoid: the NS state rows,
                              then each env's kinematics cache, AoS)             */
  int32_t* env_int;        /* [2, E]: steps in episode, episodes started         */
  double* filter_state;    /* [2, filter_doubles] ping-pong running stats        */
  double* records;         /* [2, n_blocks, record_doubles] per-block partials   */
  int64_t* iteration;      /* device iteration counter (RNG step base)           */
  float* obs;              /* [T*E, obs_dim] filtered observations (core.py:191-192) */
  void* act;               /* [T*E] int32 | [T*E, d] float                        */
  float* prob;             /* [T*E, k | 2d]                                       */
  float* rew;              /* [T*E] raw rewards (core.py:198)                     */
  uint8_t* flags;          /* [T*E] bit0 last-of-episode, bit1 terminated         */
  int32_t* ep_t;           /* [T*E] step index of the row inside its episode      */
  const void* noise;       /* sampling-noise rows (double) [T*E] u | [T*E, d] z: from
                              mrl_rollout_noise, or injected (parity tests)       */
  int64_t* stamps;         /* optional diagnostic: [T, 16] s_memrealtime of block 0 phases (NULL in production) */
  double* raw_obs;         /* layered rollout: [obs_dim+1, E] raw next obs + reward (SoA) */
  uint16_t* obs_bf16;      /* layered rollout, optional: [E, ld8(obs_dim)] the step's filtered
                              rows also as bf16 (RNE; the first hidden GEMM's operand), columns
                              obs_dim.. left as they are (caller zeroes them once); NULL: none */
} mrl_rollout_bufs;

/* env_state doubles per env (Humanoid: qpos ++ qvel ++ ctrl, 64, plus the 565-double
   kinematics cache the step kernels keep of the stored state) */
int64_t mrl_env_state_doubles(int32_t env_id);
int64_t mrl_filter_doubles(int32_t env_id);
int64_t mrl_record_doubles(int32_t env_id);
int64_t mrl_rollout_blocks(int32_t n_envs);
/* the Philox sampling noise of the CURRENT iteration (device counter b->iteration):
 * out[T*E] uniforms (Categorical) | out[T*E, d] normals (DiagGauss), row = t*E + e --
 * drawn once per iteration, before the steps, and passed as b->noise */
int64_t mrl_rollout_noise_doubles(const mrl_rollout_desc* d);
int mrl_rollout_noise(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, double* out, void* stream);
/* reset every env (start of iteration, core.py:186) and publish obs_0 partials */
int mrl_rollout_reset(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream);
/* policy image of the fused step kernel (16 envs per wave on 16x16x4 MFMA tiles,
 * mlp_layout.h rollout_dims): floats of it, and its packing from flat theta -- once
 * per iteration, before the steps (theta changes between iterations) */
int64_t mrl_rollout_image_floats(const mrl_mlp_desc* pol);
int mrl_rollout_pack(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, float* rimage,
                     void* stream);
/* one lock-step env step t (0 <= t < horizon) for all envs; rimage from mrl_rollout_pack */
int mrl_rollout_step(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta,
                     const float* rimage, const mrl_rollout_bufs* b, int32_t t, void* stream);
/* The whole horizon of the fused path in one call: reset + steps 0..T-1 (then
 * mrl_rollout_finish).  persistent != 0: ONE cooperative launch whose blocks stay
 * resident and loop over the steps, handing the per-step running-stat partials to each
 * other as step-tagged granules in sync (device workspace of mrl_rollout_sync_bytes(d)
 * bytes, zeroed by this call; the u32 sync[32] != 0 afterwards means the grid could not
 * run resident and gave up).  Falls back to mrl_rollout_reset + T x mrl_rollout_step
 * (identical results) when persistent == 0, sync is NULL, or the stream's CUs are fewer
 * than the blocks. */
int64_t mrl_rollout_sync_bytes(const mrl_rollout_desc* d);
int mrl_rollout_run(const mrl_rollout_desc* d, const mrl_mlp_desc* pol, const float* theta, const float* rimage,
                    const mrl_rollout_bufs* b, uint32_t* sync, int32_t persistent, void* stream);
/* Layered-policy rollout (any policy net; required for Humanoid): step t is
 *   mrl_rollout_obs(t)            filter merge + normalised obs rows of step t -> b->obs
 *   <policy forward over the E rows of step t, e.g. LayeredMlpNet GEMMs> -> z [E, n_out]
 *   mrl_rollout_act(z, t)         sample, env step, raw next obs/reward, block partials
 * mrl_rollout_reset_rows replaces mrl_rollout_reset; mrl_rollout_finish is shared. */
int mrl_rollout_reset_rows(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream);
int mrl_rollout_obs(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, int32_t t, void* stream);
int mrl_rollout_act(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const float* z, const float* logstd,
                    const mrl_rollout_bufs* b, int32_t t, void* stream);
/* Humanoid: the same step with the policy head fused in -- the caller's forward stops at
 * the last hidden layer (hidden [E, n_hidden]) and the step computes z = hidden . w_head
 * + b_head per env (w_head [n_hidden, n_out] Keras layout; MRL_COMPUTE_BF16 in the desc
 * rounds hidden and w_head to bf16 like the layered bf16 GEMM) */
int mrl_rollout_act_head(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const float* hidden,
                         int32_t n_hidden, const float* w_head, const float* b_head, const float* logstd,
                         const mrl_rollout_bufs* b, int32_t t, void* stream);
/* the same with the last hidden layer as bf16 rows (hidden16 [E, n_hidden] uint16 bf16
 * bits, the bf16 tape's activations from mrl_gemm_bf16): MRL_COMPUTE_BF16 only */
int mrl_rollout_act_head_bf16(const mrl_rollout_desc* d, int32_t head, int32_t n_out, const uint16_t* hidden16,
                              int32_t n_hidden, const float* w_head, const float* b_head, const float* logstd,
                              const mrl_rollout_bufs* b, int32_t t, void* stream);
/* after step T-1: fold the last reward partials into the reward stat, advance the
 * iteration counter (obs_T is never pushed: the horizon cuts the episode) */
int mrl_rollout_finish(const mrl_rollout_desc* d, const mrl_rollout_bufs* b, void* stream);

/* ---------------------------------------------------------------- streams
 * CU-masked HIP streams for the iteration pipeline (the rollout of iteration k+1
 * and the VF fit of iteration k run at once on disjoint CU sets).  No reference
 * counterpart: the reference runs single-threaded on the CPU (core.py:135-171).
 * mask: `words` 32-bit words, bit i = CU i (hipExtStreamCreateWithCUMask). */
int mrl_device_cu_count(int32_t* out);
int mrl_stream_create_cu_mask(const uint32_t* mask, int32_t words, void** stream_out);
int mrl_stream_get_cu_mask(void* stream, int32_t words, uint32_t* mask);
int mrl_stream_destroy(void* stream);
/* cross-stream ordering on a memory value: mrl_stream_signal enqueues "flag = value" on the
 * producer's stream (after its prior work), mrl_stream_wait makes the consumer's stream
 * wait until flag >= value.  flag: device memory written by one producer stream only, with
 * increasing values; the signal is enqueued before the wait. */
int mrl_stream_signal(void* stream, uint32_t* flag, uint32_t value);
int mrl_stream_wait(void* stream, uint32_t* flag, uint32_t value);

#ifdef __cplusplus
}
#endif
#endif
