"""ctypes front of oracle/mlp_c.c -- TEST INFRASTRUCTURE (oracle).

``CRows`` has the interface of ``trpo_np.RowChunks`` (pg / fvp / losses as float64 batch
means), so ``trpo_np.trpo_update(..., rows=CRows(...))`` runs the reference's
``TrpoUpdater.__call__`` orchestration (`trpo.py:72-140`) with the per-row math in C:
the float64 truth at the benchmark's 4.19 M rows in seconds.  Built by the Makefile
(``make oracle``) and ``__graft_entry__.build()``; pinned against the numpy restatement
by ``tests/test_oracle_c.py``."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmrl_oracle.so")
_lib = None
_D = ctypes.POINTER(ctypes.c_double)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} is not built (make oracle)")
        _lib = ctypes.CDLL(LIB_PATH)
        for f in ("mrlo_pg", "mrlo_fvp", "mrlo_losses"):
            getattr(_lib, f).restype = ctypes.c_int
    return _lib


def _p(a):
    return a.ctypes.data_as(_D) if a is not None else None


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


class CRows:
    def __init__(self, spec, ob, act=None, adv=None, oldprob=None, threads=16, cache=True):
        if spec.head not in ("gauss", "softmax"):
            raise ValueError("policy heads only")
        self.spec = spec
        self.n = ob.shape[0]
        self.ob, self.act, self.adv, self.oldprob = _f64(ob), _f64(act), _f64(adv), _f64(oldprob)
        self.threads = int(threads)
        self.hid = (ctypes.c_int * max(1, len(spec.hid)))(*spec.hid)
        self.args = (spec.n_in, len(spec.hid), self.hid, spec.n_out, 0 if spec.head == "gauss" else 1)
        # the primal activations of one theta, reused by the CG products of an update
        self.cache = np.empty((self.n, spec.n_in + sum(spec.hid) + spec.n_out)) if cache else None
        self.cache_key = None

    def _cache(self, theta):
        """(pointer, fill) for theta: fill on a new theta, read on a repeat"""
        if self.cache is None:
            return None, 0
        key = np.asarray(theta, dtype=np.float64).tobytes()
        if key == self.cache_key:
            return _p(self.cache), 0
        self.cache_key = key
        return _p(self.cache), 1

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"oracle C call failed ({rc})")

    def pg(self, spec, theta, dtype=np.float64):
        g = np.zeros(self.spec.P)
        self._check(lib().mrlo_pg(*self.args, _p(_f64(theta)), _p(self.ob), _p(self.act), _p(self.adv),
                                  _p(self.oldprob), ctypes.c_int64(self.n), self.threads, _p(g), *self._cache(theta)))
        return g

    def fvp(self, spec, theta, v, dtype=np.float64):
        out = np.zeros(self.spec.P)
        self._check(lib().mrlo_fvp(*self.args, _p(_f64(theta)), _p(_f64(v)), _p(self.ob), ctypes.c_int64(self.n),
                                   self.threads, _p(out), *self._cache(theta)))
        return out

    def losses(self, spec, theta, dtype=np.float64):
        out = np.zeros(3)
        self._check(lib().mrlo_losses(*self.args, _p(_f64(theta)), _p(self.ob), _p(self.act), _p(self.adv),
                                      _p(self.oldprob), ctypes.c_int64(self.n), self.threads, _p(out),
                                      *self._cache(theta)))
        return out
