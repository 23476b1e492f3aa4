"""Device MLP nets: flat fp32 theta + packed LDS image, driven through libmrl_hip.

Replaces the Keras ``Sequential`` + Theano function machinery of the reference
(`agentzoo.py:25-60`, `core.py:296-336`, `core.py:518-557`): parameters live in
one flat device vector in Keras ``trainable_weights`` order, and every pass over
a batch is one fused HIP launch (``mrl_mlp_rows`` / ``mrl_mlp_vjp``).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import MrlError, call, ptr, stream

HIDDEN = 64
N_LAYERS = 2


def check_hid_sizes(hid_sizes):
    hid = list(hid_sizes)
    if hid != [HIDDEN] * N_LAYERS:
        raise MrlError(f"hid_sizes={hid} is not implemented on the HIP path (only [64, 64]); "
                       "there is no CPU fallback")


def glorot_init(rng, n_in, n_out, head):
    """Keras glorot-uniform kernels, zero biases, last kernel x0.1, logstd 0 (`agentzoo.py:34-48`)."""
    arrs = []
    dims = [n_in] + [HIDDEN] * N_LAYERS + [n_out]
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


class MlpNet:
    """tanh MLP n_in -> 64 -> 64 -> n_out with a linear / softmax / DiagGauss head."""

    def __init__(self, n_in, n_out, head, device="cuda"):
        self.lib = _lib.load(require_gpu=True)
        self.desc = _lib.MlpDesc(n_in, n_out, head, HIDDEN, N_LAYERS)
        self.n_in, self.n_out, self.head = n_in, n_out, head
        P = self.lib.mrl_mlp_num_params(ctypes.byref(self.desc))
        if P < 0:
            raise MrlError(self.lib.mrl_last_error().decode())
        self.P = int(P)
        self.image_floats = int(self.lib.mrl_mlp_image_floats(ctypes.byref(self.desc)))
        self.device = torch.device(device)
        self.theta = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        self.image = torch.zeros(self.image_floats, dtype=torch.float32, device=self.device)
        self.gh = 2 * n_out if head == _lib.HEAD_GAUSS else n_out
        self.ws = Workspace(self.device)

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
        call("mrl_mlp_pack", ctypes.byref(self.desc), ptr(theta), ptr(image), int(fwd_only), ptr(skip), stream())

    # ---- fused passes
    def rows(self, epi, x, n, ep_t=None, timestep_limit=1.0, inv_n_global=1.0, act=None, adv=None, oldprob=None,
             target=None, out=None, ghead=None, partial=None, theta=None, image=None, tangent=None, image_t=None,
             skip=None):
        io = _lib.RowsIO(ptr(x), ptr(ep_t), float(timestep_limit), int(n), float(inv_n_global), ptr(act), ptr(adv),
                         ptr(oldprob), ptr(target), ptr(out), ptr(ghead), ptr(partial))
        theta = self.theta if theta is None else theta
        image = self.image if image is None else image
        call("mrl_mlp_rows", ctypes.byref(self.desc), int(epi), ptr(theta), ptr(image), ptr(tangent), ptr(image_t),
             ctypes.byref(io), ptr(skip), stream())

    def partial_rows(self, n):
        return int(self.lib.mrl_partial_rows(int(n)))

    def vjp_flat(self, x, n, ghead, out, ep_t=None, timestep_limit=1.0, image=None, skip=None):
        """out[P] (fp32) <- sum_n J_n^T ghead_n (per-wave slab + deterministic reduce)."""
        rows = int(self.lib.mrl_slab_rows(int(n)))
        slab = self.ws.get("slab", rows * self.P, torch.float32)
        image = self.image if image is None else image
        call("mrl_mlp_vjp", ctypes.byref(self.desc), ptr(image), ptr(x), ptr(ep_t), float(timestep_limit),
             ptr(ghead), int(n), ptr(slab), ptr(skip), stream())
        call("mrl_reduce_rows_f32", ptr(slab), rows, self.P, ptr(out), ptr(skip), stream())
        return out

    def reduce_partial(self, partial, n, out):
        rows = self.partial_rows(n)
        call("mrl_reduce_rows_f64", ptr(partial), rows, 4, ptr(out), None, stream())
        return out

    def forward(self, x, n, ep_t=None, timestep_limit=1.0, out=None):
        """prob rows (policy) or values (VF) for n rows of x."""
        width = 1 if self.head == _lib.HEAD_LINEAR else self.gh
        if out is None:
            out = torch.empty((int(n), width) if width > 1 else (int(n),), dtype=torch.float32, device=self.device)
        self.rows(_lib.EPI_PROB, x, n, ep_t=ep_t, timestep_limit=timestep_limit, out=out)
        return out
