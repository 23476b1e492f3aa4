"""Device MLP nets: flat fp32 theta driven through libmrl_hip.

Replaces the Keras ``Sequential`` + Theano function machinery of the reference
(`agentzoo.py:25-60`, `core.py:296-336`, `core.py:518-557`): parameters live in
one flat device vector in Keras ``trainable_weights`` order.  Two device
implementations share one interface (``rows`` / ``vjp_flat`` / ``forward``):

* ``MlpNet`` -- hid_sizes [64, 64], n_in <= 32, n_out <= 8 (CartPole, Hopper):
  every pass over a batch is one fused launch (``mrl_mlp_rows`` / ``mrl_mlp_vjp``)
  with the weights resident in LDS as a packed image.
* ``LayeredMlpNet`` -- any hid_sizes / widths (Humanoid 376-512-512-512-17): each
  Dense layer is one tiled MFMA GEMM over all rows (``mrl_gemm``), the head
  epilogue is ``mrl_head_rows``; the forward activations of the last recording pass
  are kept as a tape so the Fisher products of one update reuse them.

``make_net`` picks the fused path whenever the shape allows it.
"""
import contextlib
import ctypes
import os

import numpy as np
import torch

from . import _lib, timing
from ._lib import MrlError, call, ptr, stream

# GEMM launches over at least this many rows are timed one by one when bench.py enables
# timing (the update's and the VF fit's passes; not the rollout's per-step GEMMs)
GEMM_TIMING_MIN_ROWS = 1 << 16
# fp32 policy GEMMs below this many rows (the rollout's per-step forward over E rows and
# the small-M launches) run on split bf16 operands (MRL_COMPUTE_SPLIT): on the C5 rollout
# 405 -> 363 ms per iteration against the exact-f32 kernel (profiles/r05o_bench_humanoid*.json);
# the single-product NN / NT launches above it measured faster in exact f32
SPLIT_SMALL_M_ROWS = 1 << 16

HIDDEN = 64
N_LAYERS = 2


MAX_OUT_LAYERED = 32
FUSED_MAX_IN, FUSED_MAX_OUT = 32, 8


def check_hid_sizes(hid_sizes):
    hid = [int(h) for h in hid_sizes]
    if len(hid) < 1 or min(hid) < 1:
        raise MrlError(f"hid_sizes={hid}: need at least one hidden layer of positive width")
    return hid


def fused_ok(n_in, n_out, hid_sizes):
    return list(hid_sizes) == [HIDDEN] * N_LAYERS and n_in <= FUSED_MAX_IN and n_out <= FUSED_MAX_OUT


def check_dtype(dtype):
    if dtype not in _lib.COMPUTE:
        raise MrlError(f"mlp dtype {dtype!r}: expected one of {sorted(_lib.COMPUTE)}")
    return dtype


def make_net(n_in, n_out, head, hid_sizes=(HIDDEN,) * N_LAYERS, impl="auto", device="cuda", dtype="fp32"):
    """Fused 64-wide net when the shape allows it (impl="auto"), else the layered net.
    dtype: MFMA operand precision of every pass -- "fp32" (exact f32 MFMA, the parity
    dtype) or "bf16" (operands rounded to bf16, f32 accumulation: the throughput mode)."""
    hid = check_hid_sizes(hid_sizes)
    check_dtype(dtype)
    if impl not in ("auto", "fused", "layered"):
        raise MrlError(f"mlp impl {impl!r}: expected auto, fused or layered")
    if impl == "fused" or (impl == "auto" and fused_ok(n_in, n_out, hid)):
        if not fused_ok(n_in, n_out, hid):
            raise MrlError(f"fused MLP path needs hid_sizes=[64, 64], n_in<=32, n_out<=8 (got {hid}, {n_in}, {n_out})")
        return MlpNet(n_in, n_out, head, device=device, dtype=dtype)
    return LayeredMlpNet(n_in, n_out, head, hid, device=device, dtype=dtype)


def glorot_init(rng, n_in, n_out, head, hid_sizes=(HIDDEN,) * N_LAYERS):
    """Keras glorot-uniform kernels, zero biases, last kernel x0.1, logstd 0 (`agentzoo.py:34-48`)."""
    arrs = []
    dims = [n_in] + list(hid_sizes) + [n_out]
    for i in range(len(dims) - 1):
        lim = np.sqrt(6.0 / (dims[i] + dims[i + 1]))
        W = rng.uniform(-lim, lim, size=(dims[i], dims[i + 1]))
        if i == len(dims) - 2 and head != _lib.HEAD_LINEAR:
            W = W * 0.1
        arrs += [W.ravel(), np.zeros(dims[i + 1])]
    if head == _lib.HEAD_GAUSS:
        arrs.append(np.zeros(n_out))
    return np.concatenate(arrs).astype(np.float32)


class Workspace:
    """Reusable device scratch sized for a batch of n rows (grown on demand)."""

    def __init__(self, device):
        self.device = device
        self._bufs = {}

    def get(self, name, numel, dtype):
        t = self._bufs.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.empty(max(int(numel), 1), dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t[:numel]


_SPLIT_ROWS_EPIS = (_lib.EPI_PROB, _lib.EPI_LOSSES, _lib.EPI_SURRGRAD, _lib.EPI_VFLOSS)


class MlpNet:
    """tanh MLP n_in -> 64 -> 64 -> n_out with a linear / softmax / DiagGauss head."""

    layered = False

    def __init__(self, n_in, n_out, head, device="cuda", dtype="fp32"):
        self.lib = _lib.load(require_gpu=True)
        self.dtype = check_dtype(dtype)
        self.bf16 = dtype == "bf16"
        # bf16: the _bf16 entry points (csrc/mlp_bf16.hip) with their own image / cache
        self._sfx = "_bf16" if self.bf16 else ""
        self.desc = _lib.MlpDesc(n_in, n_out, head, HIDDEN, N_LAYERS)
        self.n_in, self.n_out, self.head = n_in, n_out, head
        P = self.lib.mrl_mlp_num_params(ctypes.byref(self.desc))
        if P < 0:
            raise MrlError(self.lib.mrl_last_error().decode())
        self.P = int(P)
        self.image_floats = int((self.lib.mrl_mlp_image_words_bf16 if self.bf16 else self.lib.mrl_mlp_image_floats)(
            ctypes.byref(self.desc)))
        self.device = torch.device(device)
        self.theta = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        self.image = torch.zeros(self.image_floats, dtype=torch.float32, device=self.device)
        self.gh = 2 * n_out if head == _lib.HEAD_GAUSS else n_out
        self.hid_sizes = [HIDDEN] * N_LAYERS
        self.ws = Workspace(self.device)
        # primal activation cache (h1/h2 of the last recording pass at self.theta):
        # the Fisher products of an update and the VJP after a loss pass reuse it
        self.use_cache = True
        self._cache_key = None
        # the fp32 Fisher product's JVP half on bf16 MFMA with exactly split operands
        # (csrc/mlp_split.hip): MRL_FISHER=split (default) | f32 (the exact-f32 MFMA rows kernel)
        self.fisher_split = (not self.bf16) and os.environ.get("MRL_FISHER", "split") == "split"
        # the whole Fisher product in one launch (mrl_mlp_fisher_hyb) where the shape allows
        # it; MRL_FISHER_ONEPASS=0: the split JVP rows + hybrid VJP pair
        self.fisher_onepass = (self.fisher_split and os.environ.get("MRL_FISHER_ONEPASS", "1") != "0"
                               and bool(self.lib.mrl_mlp_fisher_hyb_fits(ctypes.byref(self.desc))))
        # the forward row passes (PROB / LOSSES / SURRGRAD / VFLOSS) of the net's own theta
        # on the same split operands (mrl_mlp_rows_split); MRL_ROWS_SPLIT=0: exact-f32 kernel
        self.rows_split = self.fisher_split and os.environ.get("MRL_ROWS_SPLIT", "1") != "0"
        # the policy gradient (SURRGRAD rows + VJP) in one launch (mrl_mlp_grad_hyb), on the
        # one-pass Fisher product's shapes; MRL_GRAD_ONEPASS=0: the rows + VJP pair
        self.grad_onepass = (self.fisher_onepass and self.rows_split
                             and os.environ.get("MRL_GRAD_ONEPASS", "1") != "0")
        self.image_s = None
        if self.fisher_split:
            w = int(self.lib.mrl_mlp_image_words_split(ctypes.byref(self.desc)))
            self.image_s = torch.zeros(w, dtype=torch.float32, device=self.device)

    # ---- flat parameter plumbing (GetFlat / SetFromFlat, core.py:518-557)
    def get_flat(self):
        return self.theta.detach().cpu().numpy().copy()

    def set_flat(self, th):
        th = torch.as_tensor(np.asarray(th), dtype=torch.float32)  # SetFromFlat casts to floatX (core.py:540)
        self.theta.copy_(th.to(self.device))
        self.pack()

    def pack(self, theta=None, image=None, fwd_only=False, skip=None):
        theta = self.theta if theta is None else theta
        image = self.image if image is None else image
        if image is self.image:
            # the net's own weights change: a cached forward of the old ones is stale (raw
            # device writes to theta, e.g. mrl_adam_step, do not bump theta._version)
            self._cache_key = None
        call("mrl_mlp_pack" + self._sfx, ctypes.byref(self.desc), ptr(theta), ptr(image), int(fwd_only), ptr(skip),
             stream())
        if image is self.image and self.fisher_split:
            call("mrl_mlp_pack_split", ctypes.byref(self.desc), ptr(theta), ptr(self.image_s), ptr(skip), stream())

    def new_tangent_image(self):
        """Image buffer for Fisher-product tangents (pack_tangent): a split image when the
        Fisher products run on split operands."""
        if self.fisher_split:
            t = torch.zeros_like(self.image_s)
            t._mrl_split = True  # rows(EPI_FVP) takes the split kernel for images marked so
            return t
        return torch.zeros_like(self.image)

    def new_candidate_image(self):
        """Image buffer for a candidate theta's forward passes (pack_candidate): a split
        image (marked) when the row passes run on split operands, else an f32 image."""
        if self.rows_split:
            t = torch.zeros_like(self.image_s)
            t._mrl_split_fwd = True  # rows() takes the split kernel for images marked so
            return t
        return torch.zeros_like(self.image)

    def pack_candidate(self, theta, image, skip=None):
        if getattr(image, "_mrl_split_fwd", False):
            call("mrl_mlp_pack_split", ctypes.byref(self.desc), ptr(theta), ptr(image), ptr(skip), stream())
        else:
            self.pack(theta=theta, image=image, fwd_only=True, skip=skip)

    def pack_tangent(self, v, image, skip=None):
        if self.fisher_split:
            call("mrl_mlp_pack_split", ctypes.byref(self.desc), ptr(v), ptr(image), ptr(skip), stream())
        else:
            self.pack(theta=v, image=image, fwd_only=True, skip=skip)

    # ---- fused passes
    def rows(self, epi, x, n, ep_t=None, timestep_limit=1.0, inv_n_global=1.0, act=None, adv=None, oldprob=None,
             target=None, out=None, ghead=None, partial=None, theta=None, image=None, tangent=None, image_t=None,
             skip=None, kl_coeff=0.0, kl_cutoff=0.0, cutoff_coeff=0.0, reverse_kl=0, feat_out=None):
        own = (theta is None or theta is self.theta) and (image is None or image is self.image)
        theta = self.theta if theta is None else theta
        image = self.image if image is None else image
        mode, cache = _lib.CACHE_NONE, None
        if self.use_cache and own:
            key = self._key(x, n, ep_t, timestep_limit)
            if epi in (_lib.EPI_SURRGRAD, _lib.EPI_VFLOSS, _lib.EPI_PPOGRAD):
                mode, cache = _lib.CACHE_WRITE, self._cache(n)
                self._cache_key = key
            elif epi == _lib.EPI_FVP and self._cache_key == key:
                mode, cache = _lib.CACHE_READ, self._cache(n)
        if epi == _lib.EPI_FVP and getattr(image_t, "_mrl_split", False):
            if mode != _lib.CACHE_READ:
                # split products read the f32 activation cache; without one the tangent is
                # repacked as an f32 image for the exact-f32 kernel
                t32 = self.ws.get("tan_f32_image", self.image.numel(), torch.float32)
                self.pack(theta=tangent, image=t32, fwd_only=True, skip=skip)
                image_t = t32
            else:
                io = _lib.RowsIO(ptr(x), ptr(ep_t), float(timestep_limit), int(n), float(inv_n_global), None, None,
                                 None, None, None, ptr(ghead), None, 0.0, 0.0, 0.0, 0, mode, ptr(cache), None)
                call("mrl_mlp_fvp_split", ctypes.byref(self.desc), ptr(theta), ptr(self.image_s), ptr(tangent),
                     ptr(image_t), ctypes.byref(io), ptr(skip), stream())
                return
        io = _lib.RowsIO(ptr(x), ptr(ep_t), float(timestep_limit), int(n), float(inv_n_global), ptr(act), ptr(adv),
                         ptr(oldprob), ptr(target), ptr(out), ptr(ghead), ptr(partial), float(kl_coeff),
                         float(kl_cutoff), float(cutoff_coeff), int(reverse_kl), mode, ptr(cache), ptr(feat_out))
        if self.rows_split and epi in _SPLIT_ROWS_EPIS and (own or getattr(image, "_mrl_split_fwd", False)):
            call("mrl_mlp_rows_split", ctypes.byref(self.desc), int(epi), ptr(theta),
                 ptr(self.image_s if own else image), ctypes.byref(io), ptr(skip), stream())
            return
        call("mrl_mlp_rows" + self._sfx, ctypes.byref(self.desc), int(epi), ptr(theta), ptr(image), ptr(tangent),
             ptr(image_t), ctypes.byref(io), ptr(skip), stream())

    def _key(self, x, n, ep_t, timestep_limit):
        return (self.theta.data_ptr(), self.theta._version, x.data_ptr(), int(n),
                None if ep_t is None else ep_t.data_ptr(), float(timestep_limit))

    def _cache(self, n):
        words = (self.lib.mrl_act_cache_words_bf16 if self.bf16 else self.lib.mrl_act_cache_floats)(int(n))
        return self.ws.get("act_cache", int(words), torch.float32)

    def size_for_cus(self, cus):
        """Size the row passes' and the VJP's grids for a stream of ``cus`` CUs (0: the
        whole device): the VF fit runs beside the rollout on a CU subset, where a grid
        sized for all CUs would leave a partial second round.  The per-wave partial sums
        follow the grid, so both iteration orders set the same value (core.IterationRunner)."""
        self.desc.cus = int(cus)

    def partial_rows(self, n):
        fn = self.lib.mrl_mlp_partial_rows_bf16 if self.bf16 else self.lib.mrl_mlp_partial_rows
        return int(fn(ctypes.byref(self.desc), int(n)))

    def vjp_flat(self, x, n, ghead, out, ep_t=None, timestep_limit=1.0, image=None, skip=None):
        """out[P] (fp32) <- sum_n J_n^T ghead_n (per-wave slab + deterministic reduce); the
        forward comes from the activation cache when the last recording pass was at
        self.theta on the same rows."""
        fn = self.lib.mrl_mlp_slab_rows_bf16 if self.bf16 else self.lib.mrl_mlp_slab_rows
        rows = int(fn(ctypes.byref(self.desc), int(n)))
        slab = self.ws.get("slab", rows * self.P, torch.float32)
        cache = None
        if self.use_cache and image is None and self._cache_key == self._key(x, n, ep_t, timestep_limit):
            cache = self._cache(n)
        image = self.image if image is None else image
        call("mrl_mlp_vjp" + self._sfx, ctypes.byref(self.desc), ptr(image), ptr(x), ptr(ep_t),
             float(timestep_limit), ptr(ghead), int(n), ptr(slab), ptr(cache), ptr(skip), stream())
        call("mrl_reduce_rows_f32", ptr(slab), rows, self.P, ptr(out), ptr(skip), stream())
        return out

    def fisher_onepass_applies(self, x, n, image_t):
        return bool(self.fisher_onepass and getattr(image_t, "_mrl_split", False) and self.use_cache
                    and self._cache_key == self._key(x, n, None, 1.0))

    def fisher_product(self, x, n, inv_n_global, tangent, image_t, out, skip=None):
        """out[P] <- the Fisher product along ``tangent`` over the n cached rows in ONE
        launch (mrl_mlp_fisher_hyb: split JVP rows and hybrid VJP side by side in each
        block, the head-gradient rows through LDS) when it applies -- a split tangent image,
        a current activation cache of these rows, a shape mrl_mlp_fisher_hyb_fits accepts.
        False: not applicable (the caller runs rows(EPI_FVP) + vjp_flat)."""
        if not self.fisher_onepass_applies(x, n, image_t):
            return False
        rows = int(self.lib.mrl_mlp_slab_rows(ctypes.byref(self.desc), int(n)))
        slab = self.ws.get("slab", rows * self.P, torch.float32)
        io = _lib.RowsIO(ptr(x), None, 1.0, int(n), float(inv_n_global), None, None, None, None, None, None,
                         None, 0.0, 0.0, 0.0, 0, _lib.CACHE_READ, ptr(self._cache(n)), None)
        call("mrl_mlp_fisher_hyb", ctypes.byref(self.desc), ptr(self.theta), ptr(self.image), ptr(self.image_s),
             ptr(tangent), ptr(image_t), ctypes.byref(io), ptr(slab), ptr(skip), stream())
        call("mrl_reduce_rows_f32", ptr(slab), rows, self.P, ptr(out), ptr(skip), stream())
        return True

    def grad_onepass_applies(self, ep_t=None):
        return bool(self.grad_onepass and self.use_cache and ep_t is None)

    def policy_gradient(self, x, n, inv_n_global, act, adv, oldprob, out, sums):
        """out[P] <- the surrogate's gradient and sums[4] <- (surr, kl, ent, 0) summed over
        the n rows in ONE launch (mrl_mlp_grad_hyb: the SURRGRAD rows of
        mrl_mlp_rows_split and the hybrid VJP side by side in each block, the head-gradient
        rows through LDS), recording the activation cache as the rows pass does.  False:
        not applicable (the caller runs rows(EPI_SURRGRAD) + vjp_flat)."""
        if not self.grad_onepass_applies():
            return False
        rows = int(self.lib.mrl_mlp_slab_rows(ctypes.byref(self.desc), int(n)))
        slab = self.ws.get("slab", rows * self.P, torch.float32)
        partial = self.ws.get("grad_partial", rows * 4, torch.float64)  # one row per producer wave
        self._cache_key = self._key(x, n, None, 1.0)
        io = _lib.RowsIO(ptr(x), None, 1.0, int(n), float(inv_n_global), ptr(act), ptr(adv), ptr(oldprob), None,
                         None, None, ptr(partial), 0.0, 0.0, 0.0, 0, _lib.CACHE_WRITE, ptr(self._cache(n)), None)
        call("mrl_mlp_grad_hyb", ctypes.byref(self.desc), ptr(self.theta), ptr(self.image), ptr(self.image_s),
             ctypes.byref(io), ptr(slab), None, stream())
        call("mrl_reduce_rows_f32", ptr(slab), rows, self.P, ptr(out), None, stream())
        call("mrl_reduce_rows_f64", ptr(partial), rows, 4, ptr(sums), None, stream())
        return True

    def reduce_partial(self, partial, n, out):
        rows = self.partial_rows(n)
        call("mrl_reduce_rows_f64", ptr(partial), rows, 4, ptr(out), None, stream())
        return out

    def forward(self, x, n, ep_t=None, timestep_limit=1.0, out=None, feat_out=None):
        """prob rows (policy) or values (VF) for n rows of x.  feat_out (value nets, with
        ep_t): [n, n_in] receives the input rows [x, t / limit] the pass derives anyway."""
        width = 1 if self.head == _lib.HEAD_LINEAR else self.gh
        if out is None:
            out = torch.empty((int(n), width) if width > 1 else (int(n),), dtype=torch.float32, device=self.device)
        self.rows(_lib.EPI_PROB, x, n, ep_t=ep_t, timestep_limit=timestep_limit, out=out, feat_out=feat_out)
        return out


def layer_offsets(dims, gauss):
    """Flat-theta offsets of each Dense layer's W [d_in, d_out] and b, of logstd, and P."""
    w_off, b_off, off = [], [], 0
    for i in range(len(dims) - 1):
        w_off.append(off)
        off += dims[i] * dims[i + 1]
        b_off.append(off)
        off += dims[i + 1]
    tls = off
    return w_off, b_off, tls, off + (dims[-1] if gauss else 0)


class LayeredMlpNet:
    """tanh MLP n_in -> hid_sizes... -> n_out on the layered GEMM path (any widths).

    Flat theta layout (Keras trainable_weights order, core.py:518-557): for each Dense
    layer W [d_in, d_out] row-major then b [d_out]; DiagGauss appends logstd [n_out].
    ``image`` is a placeholder (the layered kernels read theta directly), so callers
    that pack images (HipTrpoOps) work unchanged."""

    layered = True
    SLAB_SPLITS = 64

    def __init__(self, n_in, n_out, head, hid_sizes, device="cuda", dtype="fp32"):
        self.lib = _lib.load(require_gpu=True)
        self.dtype = check_dtype(dtype)
        self.compute = _lib.COMPUTE[dtype]
        # fp32: the policy's weight-gradient (TN) and JVP (NN, two products) GEMMs and its
        # small-M rollout forward on split bf16 operands (mrl_gemm MRL_COMPUTE_SPLIT:
        # fp32-accurate, six bf16 part products per k-step), where they measured faster than
        # the exact-f32 kernel (C5: TN 4.77 -> 4.06 ms, JVP 9.44 -> 8.56 at 1 M rows; the
        # rollout 405 -> 363 ms per iteration); the single-product NN / NT GEMMs over 1 M rows
        # and the value net (its fit runs beside the rollout) measured slower on them and stay
        # exact f32 (profiles/r05o_bench_humanoid*.json).  MRL_GEMM_SPLIT=0: exact f32.
        self.split_gemms = (self.compute == _lib.COMPUTE_F32 and head != _lib.HEAD_LINEAR
                            and os.environ.get("MRL_GEMM_SPLIT", "1") != "0")
        if not 1 <= n_out <= MAX_OUT_LAYERED:
            raise MrlError(f"n_out={n_out}: the layered head supports 1..{MAX_OUT_LAYERED} outputs")
        if head == _lib.HEAD_LINEAR and n_out != 1:
            raise MrlError("linear head needs n_out=1")
        self.n_in, self.n_out, self.head = int(n_in), int(n_out), head
        self.hid_sizes = check_hid_sizes(hid_sizes)
        self.dims = [self.n_in] + self.hid_sizes + [self.n_out]
        self.w_off, self.b_off, self.tls, self.P = layer_offsets(self.dims, head == _lib.HEAD_GAUSS)
        self.device = torch.device(device)
        self.theta = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        self.image = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.gh = 2 * n_out if head == _lib.HEAD_GAUSS else n_out
        self.ws = Workspace(self.device)
        self.desc = None
        self._tape = None  # (key, X, ldx, [H_1..H_L], Z)
        # bf16 mode keeps the tape, the JVP / gradient chains and packed weight images in
        # bf16 and runs the large-M passes on the bf16-operand GEMMs (csrc/gemm_bf16.hip);
        # the rollout's per-step forward (forward_rows) stays on mrl_gemm, except the
        # Humanoid step's hidden layers (forward_hidden_rows_b16)
        # (hidden widths a multiple of 8: the bf16 rows are 16-B aligned with no padding)
        self.tape_bf16 = self.compute == _lib.COMPUTE_BF16 and all(h % 8 == 0 for h in self.hid_sizes)
        # LDS bytes per block the bf16 GEMMs may use (0: any kernel): a net whose passes run
        # co-scheduled beside the wave-per-env rollout takes the tiled kernels only, whose
        # short-lived blocks leave room for the rollout's (core.IterationRunner)
        self.lds_limit = 0
        # rows pinned by pin_input (the VF fit's features, read by every L-BFGS
        # evaluation): (x ptr, n, ep_t ptr) -> the tape's input (X, ldx) as last built
        self._pinned = None
        self._pinned_input = None

    # ---- flat parameter plumbing
    def get_flat(self):
        return self.theta.detach().cpu().numpy().copy()

    def set_flat(self, th):
        th = torch.as_tensor(np.asarray(th), dtype=torch.float32)
        self.theta.copy_(th.to(self.device))
        self._tape = None

    def pack(self, theta=None, image=None, fwd_only=False, skip=None):
        """No image on the layered path: the GEMMs read theta directly."""

    def new_tangent_image(self):
        return torch.zeros_like(self.image)

    def pack_tangent(self, v, image, skip=None):
        """No tangent image on the layered path."""

    def size_for_cus(self, cus):
        """The layered path's GEMM grids do not depend on it (no CU split is applied)."""

    def partial_rows(self, n):
        return int(self.lib.mrl_partial_rows(int(n)))

    def reduce_partial(self, partial, n, out):
        call("mrl_reduce_rows_f64", ptr(partial), self.partial_rows(n), 4, ptr(out), None, stream())
        return out

    # ---- GEMM helpers
    @staticmethod
    def _addr(t, off=0):
        return None if t is None else ctypes.c_void_p(t.data_ptr() + 4 * off)

    def _gemm(self, m, n, k, a, lda, b, ldb, c, ldc, a_trans=0, b_trans=0, epi=0, a2=None, b2=None, bias=None,
              h=None, ldh=0, ones_row=0, splits=1, slab_stride=0, skip=None):
        compute = self.compute
        if self.split_gemms and (a_trans or a2 is not None or max(m, k) < SPLIT_SMALL_M_ROWS):
            compute = _lib.COMPUTE_SPLIT
        g = _lib.GemmDesc(m=m, n=n, k=k, a=a, lda=lda, a_trans=a_trans, ones_row=ones_row, b=b, ldb=ldb,
                          b_trans=b_trans, epilogue=epi, a2=a2, b2=b2, c=c, ldc=ldc, bias=bias, h=h, ldh=ldh,
                          splits=splits, slab_stride=slab_stride, compute=compute)
        if timing.enabled() and max(m, k) >= GEMM_TIMING_MIN_ROWS:
            # algorithmic work of the launch: 2mnk per product; bytes = f32 operands read
            # once, C written once (SLAB: one [m, n] slab per K split), H read (DTANH)
            prods = 2 if a2 is not None else 1
            S = int(self.lib.mrl_gemm_slab_splits(k, splits)) if epi == _lib.GEMM_SLAB else 1
            nbytes = 4 * (prods * (m * k + k * n) + S * m * n + (m * n if epi == _lib.GEMM_DTANH else 0))
            kind = "TN" if a_trans else ("NT" if b_trans else ("NN_dual" if a2 is not None else "NN"))
            mode = "split" if compute == _lib.COMPUTE_SPLIT else "f32"
            timing.region(f"gemm:{mode}:{kind}:{m}x{n}x{k}", call, "mrl_gemm", ctypes.byref(g), ptr(skip), stream(),
                          flop=2 * prods * m * n * k, bytes=nbytes, kernel="gemm_f32_kernel",
                          dtype="split" if mode == "split" else "fp32")
            return
        call("mrl_gemm", ctypes.byref(g), ptr(skip), stream())

    def _input(self, x, n, ep_t, timestep_limit, name="x_time", out=None):
        """(X, ldx): obs rows, or [obs, t/limit] materialised for a value net (into
        ``out`` when given)."""
        if ep_t is None:
            return x, self.n_in
        X = self.ws.get(name, n * self.n_in, torch.float32) if out is None else out
        call("mrl_concat_time", ptr(x), ptr(ep_t), int(n), self.n_in - 1, float(timestep_limit), ptr(X), 0, stream())
        return X, self.n_in

    def _forward(self, X, ldx, n, theta, bufs, zbuf, skip=None):
        """H_l = tanh(H_{l-1} W + b) ... Z = H_L W + b into bufs[l] / zbuf."""
        L = len(self.dims) - 1
        a, lda = self._addr(X), ldx
        for l in range(L):
            din, dout = self.dims[l], self.dims[l + 1]
            last = l == L - 1
            out = zbuf if last else bufs[l]
            self._gemm(n, dout, din, a, lda, self._addr(theta, self.w_off[l]), dout, self._addr(out), dout,
                       epi=_lib.GEMM_STORE if last else _lib.GEMM_TANH, bias=self._addr(theta, self.b_off[l]),
                       skip=skip)
            a, lda = self._addr(out), dout

    def _key(self, theta, x, n, ep_t):
        return (theta.data_ptr(), theta._version, x.data_ptr(), int(n), None if ep_t is None else ep_t.data_ptr())

    # ---- bf16 tape path
    @staticmethod
    def _ld8(d):
        return (int(d) + 7) // 8 * 8

    def _bf(self, name, rows, ld):
        return self.ws.get(name, int(rows) * int(ld), torch.int16)

    def _pack_images(self, vec, tag, transpose):
        """bf16 images of the Dense kernels in flat vector `vec`: transpose 1 -> W^T
        [dout, ld8(din)] (the B operand of X.W), 0 -> W [din, ld8(dout)] (of G.W^T)."""
        out = []
        for l in range(len(self.dims) - 1):
            din, dout = self.dims[l], self.dims[l + 1]
            rows, ld = (dout, self._ld8(din)) if transpose else (din, self._ld8(dout))
            img = self._bf(f"{tag}{l}", rows, ld)
            call("mrl_pack_w_bf16", self._addr(vec, self.w_off[l]), din, dout, int(transpose), ptr(img), ld, stream())
            out.append((img, ld))
        return out

    def _cast_rows(self, x, n, cols, ldx, name):
        ld = self._ld8(cols)
        y = self._bf(name, n, ld)
        call("mrl_cast_rows_bf16", ptr(x), int(n), int(cols), int(ldx), ptr(y), ld, stream())
        return y, ld

    def _gemm_b16(self, m, n, k, a, lda, bt, ldb, c, ldc, c_bf16, epi, a2=None, bt2=None, bias=None, h=None, ldh=0,
                  skip=None):
        g = _lib.GemmBf16Desc(m=m, n=n, k=k, a=ptr(a), lda=lda, bt=ptr(bt), ldb=ldb, a2=ptr(a2), bt2=ptr(bt2),
                              c=ptr(c), ldc=ldc, c_bf16=int(c_bf16), epilogue=epi, bias=bias, h=ptr(h), ldh=ldh,
                              lds_limit=self.lds_limit)
        if timing.enabled() and m >= GEMM_TIMING_MIN_ROWS:
            prods = 2 if a2 is not None else 1
            nbytes = 2 * prods * (m * k + n * k) + (2 if c_bf16 else 4) * m * n + (2 * m * n if h is not None else 0)
            kind = ("NN_dual" if a2 is not None else "NN") + {_lib.GEMM_TANH: "_tanh", _lib.GEMM_DTANH: "_dtanh"}.get(
                epi, "")
            timing.region(f"gemm:bf16:{kind}:{m}x{n}x{k}", call, "mrl_gemm_bf16", ctypes.byref(g), ptr(skip), stream(),
                          flop=2 * prods * m * n * k, bytes=nbytes, kernel="mrl_gemm_bf16", dtype="bf16")
            return
        call("mrl_gemm_bf16", ctypes.byref(g), ptr(skip), stream())

    def _forward_b16(self, Xb, ldx, n, theta, bufs, zbuf, skip=None):
        """H_l = bf16(tanh(H_{l-1} W + b)) ... Z = H_L W + b (f32)."""
        L = len(self.dims) - 1
        wt = self._pack_images(theta, "wt", 1)
        a, lda = Xb, ldx
        for l in range(L):
            din, dout = self.dims[l], self.dims[l + 1]
            last = l == L - 1
            out = zbuf if last else bufs[l]
            self._gemm_b16(n, dout, din, a, lda, wt[l][0], wt[l][1], out, dout, not last,
                           _lib.GEMM_STORE if last else _lib.GEMM_TANH, bias=self._addr(theta, self.b_off[l]),
                           skip=skip)
            a, lda = out, dout

    @contextlib.contextmanager
    def pin_input(self, x, n, ep_t=None):
        """While open, the caller promises that rows x[:n] (and ep_t) do not change: the
        tape's input -- [obs, t/limit] and its bf16 cast -- is built once for every
        recording pass over them instead of once per pass (the VF fit's evaluations)."""
        self._pinned = (x.data_ptr(), int(n), None if ep_t is None else ep_t.data_ptr())
        self._pinned_input = None
        try:
            yield self
        finally:
            self._pinned = None
            self._pinned_input = None

    def _tape_input(self, x, n, ep_t, timestep_limit):
        pin = self._pinned == (x.data_ptr(), int(n), None if ep_t is None else ep_t.data_ptr())
        if pin and self._pinned_input is not None:
            return self._pinned_input
        X, ldx = self._input(x, n, ep_t, timestep_limit, name="tape_x")
        if self.tape_bf16:
            X, ldx = self._cast_rows(X, n, self.n_in, ldx, "tape_xb")
        if pin:
            self._pinned_input = (X, ldx)
        return X, ldx

    def _record(self, x, n, ep_t, timestep_limit, theta):
        """Forward pass at theta kept as the tape the next vjp_flat / FVP uses."""
        key = self._key(theta, x, n, ep_t)
        if self.tape_bf16:
            Xb, ldxb = self._tape_input(x, n, ep_t, timestep_limit)
            H = [self._bf(f"tape_h{l}", n, d) for l, d in enumerate(self.hid_sizes)]
            Z = self.ws.get("tape_z", n * self.n_out, torch.float32)
            self._forward_b16(Xb, ldxb, n, theta, H, Z)
            self._tape = (key, Xb, ldxb, H, Z, theta)
            return self._tape
        X, ldx = self._tape_input(x, n, ep_t, timestep_limit)
        H = [self.ws.get(f"tape_h{l}", n * d, torch.float32) for l, d in enumerate(self.hid_sizes)]
        Z = self.ws.get("tape_z", n * self.n_out, torch.float32)
        self._forward(X, ldx, n, theta, H, Z)
        self._tape = (key, X, ldx, H, Z, theta)
        return self._tape

    def _scratch(self, n):
        w = max(self.hid_sizes)
        return [self.ws.get(f"scr{i}", n * w, torch.float32) for i in range(2)]

    def rows(self, epi, x, n, ep_t=None, timestep_limit=1.0, inv_n_global=1.0, act=None, adv=None, oldprob=None,
             target=None, out=None, ghead=None, partial=None, theta=None, image=None, tangent=None, image_t=None,
             skip=None, kl_coeff=0.0, kl_cutoff=0.0, cutoff_coeff=0.0, reverse_kl=0, feat_out=None):
        n = int(n)
        if feat_out is not None and (epi != _lib.EPI_PROB or ep_t is None):
            raise MrlError("feat_out is for the value prediction (EPI_PROB with ep_t)")
        theta = self.theta if theta is None else theta
        io = _lib.RowsIO(ptr(x), ptr(ep_t), float(timestep_limit), n, float(inv_n_global), ptr(act), ptr(adv),
                         ptr(oldprob), ptr(target), ptr(out), ptr(ghead), ptr(partial), float(kl_coeff),
                         float(kl_cutoff), float(cutoff_coeff), int(reverse_kl))
        dz = None
        if epi == _lib.EPI_FVP:
            if tangent is None:
                raise MrlError("EPI_FVP needs a tangent")
            tape = self._tape
            if tape is None or tape[0] != self._key(theta, x, n, ep_t):
                tape = self._record(x, n, ep_t, timestep_limit, theta)
            _, X, ldx, H, Z, _ = tape
            dz = self.ws.get("tape_dz", n * self.n_out, torch.float32)
            self._jvp(X, ldx, n, theta, tangent, H, dz, skip)
        elif epi in (_lib.EPI_SURRGRAD, _lib.EPI_VFLOSS, _lib.EPI_PPOGRAD, _lib.EPI_PPOSGD):
            _, X, ldx, H, Z, _ = self._record(x, n, ep_t, timestep_limit, theta)
        else:
            if n == 0:
                return
            X, ldx = self._input(x, n, ep_t, timestep_limit, out=feat_out)
            Z = self.ws.get("fwd_z", n * self.n_out, torch.float32)
            if self.tape_bf16:
                Xb, ldxb = self._cast_rows(X, n, self.n_in, ldx, "fwd_xb")
                w = max(self.hid_sizes)
                bufs = [self._bf(f"scrb{l % 2}", n, w) for l in range(len(self.hid_sizes))]
                self._forward_b16(Xb, ldxb, n, theta, bufs, Z, skip)
            else:
                s0, s1 = self._scratch(n)
                bufs = [s0 if l % 2 == 0 else s1 for l in range(len(self.hid_sizes))]
                self._forward(X, ldx, n, theta, bufs, Z, skip)
        gauss = self.head == _lib.HEAD_GAUSS
        call("mrl_head_rows", int(self.head), self.n_out, int(epi), ptr(Z), ptr(dz),
             self._addr(theta, self.tls) if gauss else None,
             self._addr(tangent, self.tls) if (gauss and tangent is not None) else None,
             ctypes.byref(io), ptr(skip), stream())

    def _jvp(self, X, ldx, n, theta, tangent, H, dz, skip):
        """dH_1 = (X dW0 + db0)(1-H_1^2); dH_l = (dH W + H dW + db)(1-H_l^2); dZ = dH_L W + H_L dW + db."""
        L = len(self.dims) - 1
        if self.tape_bf16:
            wt = self._pack_images(theta, "wt", 1)
            dwt = self._pack_images(tangent, "dwt", 1)
            w = max(self.hid_sizes)
            prev = None
            for l in range(L):
                din, dout = self.dims[l], self.dims[l + 1]
                last = l == L - 1
                outb = dz if last else self._bf(f"jvpb{l % 2}", n, w)
                epi = _lib.GEMM_STORE if last else _lib.GEMM_DTANH
                db = self._addr(tangent, self.b_off[l])
                h = None if last else H[l]
                if l == 0:
                    self._gemm_b16(n, dout, din, X, ldx, dwt[0][0], dwt[0][1], outb, dout, not last, epi, bias=db,
                                   h=h, ldh=dout, skip=skip)
                else:
                    self._gemm_b16(n, dout, din, prev, din, wt[l][0], wt[l][1], outb, dout, not last, epi,
                                   a2=H[l - 1], bt2=dwt[l][0], bias=db, h=h, ldh=dout, skip=skip)
                prev = outb
            return
        scr = self._scratch(n)
        prev_d = None  # dH of the previous layer
        for l in range(L):
            din, dout = self.dims[l], self.dims[l + 1]
            last = l == L - 1
            outb = dz if last else scr[l % 2]
            epi = _lib.GEMM_STORE if last else _lib.GEMM_DTANH
            W = self._addr(theta, self.w_off[l])
            dW = self._addr(tangent, self.w_off[l])
            db = self._addr(tangent, self.b_off[l])
            h = None if last else self._addr(H[l])
            if l == 0:
                self._gemm(n, dout, din, self._addr(X), ldx, dW, dout, self._addr(outb), dout, epi=epi, bias=db,
                           h=h, ldh=dout, skip=skip)
            else:
                self._gemm(n, dout, din, self._addr(prev_d), din, W, dout, self._addr(outb), dout, epi=epi,
                           a2=self._addr(H[l - 1]), b2=dW, bias=db, h=h, ldh=dout, skip=skip)
            prev_d = outb

    def vjp_flat(self, x, n, ghead, out, ep_t=None, timestep_limit=1.0, image=None, skip=None):
        """out[P] (fp32) <- sum_n J_n^T ghead_n at the tape's theta (split-K slabs + fixed-order reduce)."""
        n = int(n)
        tape = self._tape
        if tape is None or tape[0][2:] != (x.data_ptr(), n, None if ep_t is None else ep_t.data_ptr()):
            raise MrlError("LayeredMlpNet.vjp_flat needs a preceding recording rows() pass on the same rows")
        _, X, ldx, H, Z, theta = tape
        S = int(self.lib.mrl_gemm_slab_splits(n, self.SLAB_SPLITS))
        slab = self.ws.get("slab", S * self.P, torch.float32)
        L = len(self.dims) - 1
        if self.tape_bf16:
            self._vjp_b16(X, ldx, H, theta, n, ghead, slab, S, skip)
            call("mrl_reduce_rows_f32", ptr(slab), S, self.P, ptr(out), ptr(skip), stream())
            return out
        scr = self._scratch(n)
        G, ldg = ghead, self.gh
        for l in reversed(range(L)):
            din, dout = self.dims[l], self.dims[l + 1]
            inp = X if l == 0 else H[l - 1]
            # dW = inp^T G (K = rows, split over S slabs).  db rides the GEMM as a ones-row
            # when that row fits the last 128-row tile, else it is a column-sum pass.
            ones = din % 128 != 0
            self._gemm(din + ones, dout, n, self._addr(inp), din if l else ldx, self._addr(G), ldg,
                       self._addr(slab, self.w_off[l]), dout, a_trans=1, epi=_lib.GEMM_SLAB, ones_row=int(ones),
                       splits=self.SLAB_SPLITS, slab_stride=self.P, skip=skip)
            if not ones:
                call("mrl_colsum", self._addr(G), n, dout, ldg, S, self._addr(slab, self.b_off[l]), self.P, ptr(skip),
                     stream())
            if l > 0:
                Gn = scr[l % 2]
                self._gemm(n, din, dout, self._addr(G), ldg, self._addr(theta, self.w_off[l]), dout,
                           self._addr(Gn), din, b_trans=1, epi=_lib.GEMM_DTANH, h=self._addr(H[l - 1]), ldh=din,
                           skip=skip)
                G, ldg = Gn, din
        if self.head == _lib.HEAD_GAUSS:
            A = self.n_out
            call("mrl_colsum", self._addr(ghead, A), n, A, self.gh, S, self._addr(slab, self.tls), self.P, ptr(skip),
                 stream())
        call("mrl_reduce_rows_f32", ptr(slab), S, self.P, ptr(out), ptr(skip), stream())
        return out

    def _vjp_b16(self, Xb, ldx, H, theta, n, ghead, slab, S, skip):
        """The bf16 VJP: per layer the weight + bias gradient as split-K slabs (the bias as
        the ones-column of the TN GEMM) and the input gradient (G W^T)(1 - H^2) in bf16."""
        L = len(self.dims) - 1
        w_img = self._pack_images(theta, "wn", 0)
        G, ldg = self._cast_rows(ghead, n, self.gh, self.gh, "vjp_g0")
        wmax = max(self.hid_sizes)
        for l in reversed(range(L)):
            din, dout = self.dims[l], self.dims[l + 1]
            inp, lda = (Xb, ldx) if l == 0 else (H[l - 1], din)
            g = _lib.GemmBf16TnDesc(m=din + 1, n=dout, k=n, a=ptr(inp), lda=lda, b=ptr(G), ldb=ldg, ones_row=1,
                                    splits=self.SLAB_SPLITS, slab=self._addr(slab, self.w_off[l]),
                                    slab_stride=self.P, ldc=dout, lds_limit=self.lds_limit)
            if timing.enabled() and n >= GEMM_TIMING_MIN_ROWS:
                timing.region(f"gemm:bf16:TN:{din + 1}x{dout}x{n}", call, "mrl_gemm_bf16_tn", ctypes.byref(g),
                              ptr(skip), stream(), flop=2 * (din + 1) * dout * n,
                              bytes=2 * n * (lda + ldg) + 4 * S * (din + 1) * dout, kernel="mrl_gemm_bf16_tn",
                              dtype="bf16")
            else:
                call("mrl_gemm_bf16_tn", ctypes.byref(g), ptr(skip), stream())
            if l > 0:
                Gn = self._bf(f"vjpb{l % 2}", n, wmax)
                self._gemm_b16(n, din, dout, G, ldg, w_img[l][0], w_img[l][1], Gn, din, True, _lib.GEMM_DTANH,
                               h=H[l - 1], ldh=din, skip=skip)
                G, ldg = Gn, din
        if self.head == _lib.HEAD_GAUSS:
            A = self.n_out
            call("mrl_colsum", self._addr(ghead, A), n, A, self.gh, S, self._addr(slab, self.tls), self.P, ptr(skip),
                 stream())

    def forward_hidden_rows(self, x, n, bufs):
        """The hidden layers only, for a step kernel that applies the head itself; returns
        the buffer holding the last hidden layer's rows [n, hid_sizes[-1]]."""
        L = len(self.dims) - 1
        a, lda = self._addr(x), self.n_in
        out = None
        for l in range(L - 1):
            din, dout = self.dims[l], self.dims[l + 1]
            out = bufs[l % 2]
            self._gemm(int(n), dout, din, a, lda, self._addr(self.theta, self.w_off[l]), dout, self._addr(out), dout,
                       epi=_lib.GEMM_TANH, bias=self._addr(self.theta, self.b_off[l]))
            a, lda = self._addr(out), dout
        return out

    def rollout_images(self):
        """bf16 W^T images of theta for forward_hidden_rows_b16 (packed once per collect,
        inside its captured graph, so every replay sees the current policy)."""
        return self._pack_images(self.theta, "rwt", 1)

    def forward_hidden_rows_b16(self, x, n, wt, bufs16, xb, cast=True):
        """forward_hidden_rows on the bf16 tape's kernels (bf16 tape mode): obs rows cast
        to bf16 into xb (cast=False: xb already holds them), the hidden layers by
        mrl_gemm_bf16 into the bf16 row buffers bufs16 (the values the f32 path rounds at
        staging); returns the last one."""
        L = len(self.dims) - 1
        ldx = self._ld8(self.n_in)
        if cast:
            call("mrl_cast_rows_bf16", ptr(x), int(n), self.n_in, self.n_in, ptr(xb), ldx, stream())
        a, lda, out = xb, ldx, None
        for l in range(L - 1):
            din, dout = self.dims[l], self.dims[l + 1]
            out = bufs16[l % 2]
            self._gemm_b16(int(n), dout, din, a, lda, wt[l][0], wt[l][1], out, dout, True, _lib.GEMM_TANH,
                           bias=self._addr(self.theta, self.b_off[l]))
            a, lda = out, dout
        return out

    def forward_rows(self, x, n, z, bufs):
        """Head pre-activations z [n, n_out] of n obs rows into caller-owned buffers
        (the rollout's per-step forward; bufs: 2 x [n * max(hid)] scratch)."""
        hb = [bufs[l % 2] for l in range(len(self.hid_sizes))]
        self._forward(x, self.n_in, int(n), self.theta, hb, z)

    def forward(self, x, n, ep_t=None, timestep_limit=1.0, out=None, feat_out=None):
        width = 1 if self.head == _lib.HEAD_LINEAR else self.gh
        if out is None:
            out = torch.empty((int(n), width) if width > 1 else (int(n),), dtype=torch.float32, device=self.device)
        self.rows(_lib.EPI_PROB, x, n, ep_t=ep_t, timestep_limit=timestep_limit, out=out, feat_out=feat_out)
        return out
