"""Trust Region Policy Optimization update on device (`trpo.py:12-200` of the reference).

``TrpoUpdater(stochpol, usercfg)`` keeps the reference constructor, ``options``
and ``__call__(paths) -> OrderedDict(surr/kl/ent _before/_after)``; it also
exposes ``update(batch)`` on the device-resident batch of the lock-step
collector.  The numerics run in libmrl_hip:

  g, losses_before      one fused pass   (mrl_mlp_rows SURRGRAD + mrl_mlp_vjp)
  cg(F + damping I, -g) device CG vectors (fp64), 10 x [Fvp kernels + cg_update];
                        the residual-tolerance break is a device flag that turns
                        the remaining Fvp launches into no-ops (no host sync)
  shs / lm / fullstep   mrl_trpo_step_ax: shs = .5 x.(F + damping I)x where
                        (F + damping I)x = sum_k v_k z_k is accumulated by the CG
                        updates (z_k = the damped Fisher product of p_k; linearity),
                        so the Fvp(stepdir) of trpo.py:119-122 costs no pass over the
                        rows (the duplicate diagnostic Fvp of trpo.py:111 is dropped)
  linesearch            candidates theta = theta_old + frac*fullstep (fp64, cast to
                        fp32 like SetFromFlat) scored in batches (mrl_linesearch_eval:
                        K candidates, one readback / one [K, 4] all-reduce per batch;
                        batches of 1, 3 and 6 cover the reference's 10 backtracks), the
                        first accepted k in order exactly as the serial loop; the
                        accepted candidate's (surr, kl, ent) are losses_after.

In data-parallel mode every sum above is all-reduced over ranks (dist.Comm)
before it is used, so all ranks take the identical step.
"""
import ctypes
from collections import OrderedDict

import numpy as np
import torch

from . import _lib, timing
from ._lib import call, ptr, stream
from .dist import Comm
from .misc_utils import update_default_config


class HipTrpoOps:
    """The device kernels the updater drives (one policy net, one bound batch)."""

    def __init__(self, net):
        self.net = net
        P, dev = net.P, net.device
        self.P = P
        f32 = dict(dtype=torch.float32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        self.g = torch.zeros(P, **f32)
        self.fv = torch.zeros(P, **f32)
        self.b = torch.zeros(P, **f64)
        self.x = torch.zeros(P, **f64)
        self.ax = torch.zeros(P, **f64)
        self.r = torch.zeros(P, **f64)
        self.p = torch.zeros(P, **f64)
        self.p32 = torch.zeros(P, **f32)
        self.fullstep = torch.zeros(P, **f64)
        self.cand = torch.zeros(P, **f32)
        self.cand_image = (net.new_candidate_image() if hasattr(net, "new_candidate_image")
                           else torch.zeros_like(net.image))
        self.tan_image = net.new_tangent_image()
        # the CG update writes the next tangent's split image itself (mrl_cg_update_pack):
        # the Fisher product then skips its pack launch
        self.cg_pack = getattr(net, "fisher_split", False) and P <= 8192
        self._tan_packed = False
        ns = int(_lib.load().mrl_cg_state_doubles(self.P))  # scalars + block partials (wide nets)
        self.state = torch.zeros(ns, **f64)
        self.flag = torch.zeros(2, dtype=torch.int32, device=dev)
        self.step_out = torch.zeros(ns, **f64)
        self.sums = torch.zeros(4, **f64)
        self.batch = None
        self._ls = None  # batched line search: (K, candidates [K, P], images, partials, sums [K, 4])

    def bind(self, batch, inv_n_global):
        self.batch = batch
        self.inv_ng = float(inv_n_global)
        n = batch.n
        self.ghead = self.net.ws.get("ghead", n * self.net.gh, torch.float32)
        self.partial = self.net.ws.get("partial", self.net.partial_rows(n) * 4, torch.float64)

    def surrgrad(self):
        b, net = self.batch, self.net
        if getattr(net, "grad_onepass", False):
            timing.start("pg_onepass", detail=True)
            done = net.policy_gradient(b.obs, b.n, self.inv_ng, b.act, b.adv, b.prob, self.g, self.sums)
            timing.stop("pg_onepass")
            if done:
                return self.g, self.sums
        net.rows(_lib.EPI_SURRGRAD, b.obs, b.n, inv_n_global=self.inv_ng, act=b.act, adv=b.adv, oldprob=b.prob,
                 ghead=self.ghead, partial=self.partial)
        net.reduce_partial(self.partial, b.n, self.sums)
        timing.start("pg_vjp", detail=True)
        net.vjp_flat(b.obs, b.n, self.ghead, self.g)
        timing.stop("pg_vjp")
        return self.g, self.sums

    def losses(self, theta):
        b, net = self.batch, self.net
        if hasattr(net, "pack_candidate"):
            net.pack_candidate(theta, self.cand_image)
        else:
            net.pack(theta=theta, image=self.cand_image, fwd_only=True)
        net.rows(_lib.EPI_LOSSES, b.obs, b.n, inv_n_global=self.inv_ng, act=b.act, adv=b.adv, oldprob=b.prob,
                 partial=self.partial, theta=theta, image=self.cand_image)
        return net.reduce_partial(self.partial, b.n, self.sums)

    def fvp(self, v32, skip=None):
        b, net = self.batch, self.net
        if not (self._tan_packed and v32 is self.p32):
            net.pack_tangent(v32, self.tan_image, skip=skip)
            self._tan_packed = v32 is self.p32
        if getattr(net, "fisher_onepass", False) and net.fisher_onepass_applies(b.obs, b.n, self.tan_image):
            # the whole product in one launch (JVP rows and VJP side by side per block)
            timing.start("fvp_onepass", detail=True)
            net.fisher_product(b.obs, b.n, self.inv_ng, v32, self.tan_image, self.fv, skip=skip)
            timing.stop("fvp_onepass")
            return self.fv
        timing.start("fvp_jvp_rows", detail=True)
        net.rows(_lib.EPI_FVP, b.obs, b.n, inv_n_global=self.inv_ng, ghead=self.ghead, tangent=v32,
                 image_t=self.tan_image, skip=skip)
        timing.stop("fvp_jvp_rows")
        timing.start("fvp_vjp", detail=True)
        net.vjp_flat(b.obs, b.n, self.ghead, self.fv, skip=skip)
        timing.stop("fvp_vjp")
        return self.fv

    def neg_g64(self, g):
        call("mrl_cast_scale_f32_f64", ptr(g), -1.0, self.P, ptr(self.b), stream())
        return self.b

    def cg_init(self, b):
        call("mrl_cg_init", ptr(b), self.P, ptr(self.x), ptr(self.r), ptr(self.p), ptr(self.p32), ptr(self.ax),
             ptr(self.state), ptr(self.flag), stream())
        self._tan_packed = False

    def cg_update(self, fv, damping, tol):
        if self.cg_pack:
            call("mrl_cg_update_pack", ptr(fv), float(damping), float(tol), self.P, ptr(self.x), ptr(self.r),
                 ptr(self.p), ptr(self.p32), ptr(self.ax), ptr(self.state), ptr(self.flag),
                 ctypes.byref(self.net.desc), ptr(self.tan_image), stream())
            self._tan_packed = True
            return
        call("mrl_cg_update", ptr(fv), float(damping), float(tol), self.P, ptr(self.x), ptr(self.r), ptr(self.p),
             ptr(self.p32), ptr(self.ax), ptr(self.state), ptr(self.flag), stream())
        self._tan_packed = False

    def trpo_step(self, g, max_kl):
        """shs / lm / fullstep from the A x the CG updates accumulated (trpo.py:119-124)."""
        call("mrl_trpo_step_ax", ptr(self.ax), ptr(self.x), ptr(g), float(max_kl), self.P, ptr(self.fullstep),
             ptr(self.step_out), stream())
        return self.step_out

    def candidate(self, theta_old, frac):
        call("mrl_axpy_cast", ptr(theta_old), ptr(self.fullstep), float(frac), self.P, ptr(self.cand), stream())
        return self.cand

    def _ls_bufs(self, K):
        net, n = self.net, self.batch.n
        prow = net.partial_rows(n) * 4
        if self._ls is None or self._ls[0] < K or self._ls[3].shape[1] < prow:
            Kc = max(K, self._ls[0] if self._ls is not None else 0)
            dev = net.device
            iw = max(net.image.numel(), net.image_s.numel() if getattr(net, "rows_split", False) else 0)
            imgs = (torch.zeros(Kc, iw, dtype=torch.float32, device=dev)
                    if not getattr(net, "layered", False) else None)
            self._ls = (Kc, torch.zeros(Kc, self.P, dtype=torch.float32, device=dev), imgs,
                        torch.zeros(Kc, prow, dtype=torch.float64, device=dev),
                        torch.zeros(Kc, 4, dtype=torch.float64, device=dev))
        return self._ls

    def losses_batch(self, theta_old, k0, K):
        """(surr, kl, ent, n) sums of the K candidates theta_old + .5^(k0+k) fullstep
        (trpo.py:149-150) as a device [K, 4] tensor: one call on the fused path
        (mrl_linesearch_eval), candidates + K loss passes on the layered one."""
        b, net = self.batch, self.net
        _, cand, imgs, partials, sums = self._ls_bufs(K)
        if not getattr(net, "layered", False):
            io = _lib.RowsIO(ptr(b.obs), None, 1.0, int(b.n), float(self.inv_ng), ptr(b.act), ptr(b.adv), ptr(b.prob),
                             None, None, None, None, 0.0, 0.0, 0.0, 0, _lib.CACHE_NONE, None)
            compute = _lib.COMPUTE_SPLIT if getattr(net, "rows_split", False) else _lib.COMPUTE[net.dtype]
            call("mrl_linesearch_eval", ctypes.byref(net.desc), compute, ptr(theta_old),
                 ptr(self.fullstep), int(k0), int(K), ctypes.byref(io), ptr(cand), ptr(imgs), int(imgs.shape[1]),
                 ptr(partials), int(partials.shape[1]), ptr(sums), stream())
        else:
            call("mrl_linesearch_candidates", ptr(theta_old), ptr(self.fullstep), int(k0), int(K), self.P, ptr(cand),
                 stream())
            for k in range(K):
                th = cand[k]
                net.pack(theta=th, image=self.cand_image, fwd_only=True)
                net.rows(_lib.EPI_LOSSES, b.obs, b.n, inv_n_global=self.inv_ng, act=b.act, adv=b.adv, oldprob=b.prob,
                         partial=self.partial, theta=th, image=self.cand_image)
                net.reduce_partial(self.partial, b.n, sums[k])
        return sums[:K], cand


def _losses(sums, n_glob):
    s = sums.detach().double().cpu().numpy() if torch.is_tensor(sums) else np.asarray(sums, dtype=np.float64)
    return np.array([-s[0] / n_glob, s[1] / n_glob, s[2] / n_glob])


def linesearch(f, fval, expected_improve_rate, max_backtracks=10, accept_ratio=.1, trace=None):
    """Backtracking line search on the surrogate only (`trpo.py:143-159`).
    ``fval`` is the surrogate at x (the reference's ``f(x)``); ``f(stepfrac) ->
    (newfval, aux)`` evaluates the candidate x + stepfrac*fullstep on device.
    ``trace`` (a list) receives (stepfrac, actual, expected, ratio) per backtrack.
    Returns (success, stepfrac or None, k, aux)."""
    for k, stepfrac in enumerate(.5 ** np.arange(max_backtracks)):
        newfval, aux = f(stepfrac)
        actual_improve = fval - newfval
        expected_improve = expected_improve_rate * stepfrac
        ratio = actual_improve / expected_improve
        if trace is not None:
            trace.append((stepfrac, actual_improve, expected_improve, ratio))
        if ratio > accept_ratio and actual_improve > 0:
            return True, stepfrac, k, aux
    return False, None, -1, None


class TrpoUpdater:
    options = [
        ("cg_damping", float, 1e-3, "Add multiple of the identity to Fisher matrix during CG"),
        ("max_kl", float, 1e-2, "KL divergence between old and new policy (averaged over state-space)"),
    ]
    CG_ITERS = 10
    RESIDUAL_TOL = 1e-10
    MAX_BACKTRACKS = 10
    # candidates scored per readback: the first batch is k = 0 alone (accepted in most
    # updates), then 3, then the remaining 6; None: the serial one-candidate loop
    LS_BATCHES = (1, 3, 6)

    def __init__(self, stochpol, usercfg, comm=None, ops=None):
        self.cfg = update_default_config(self.options, usercfg)
        self.stochpol = stochpol
        self.comm = comm if comm is not None else Comm()
        self.ops = ops if ops is not None else HipTrpoOps(stochpol.net)
        self.loss_names = ["surr", "kl", "ent"]
        self.last_diag = {}
        # set by core.IterationRunner: called once theta is final (before its packed images,
        # which the rollout does not read), so the next iteration's rollout is issued before
        # the stats / host bookkeeping
        self.after_theta = None
        # set by core.IterationRunner: device work that may run while the host waits for
        # the update's readback (the next rollout's noise fill); issued after the copy
        self.before_readback = None
        self._host_buf = None

    def _readback(self, dev):
        """dev (float64, 1-D) to the host through a pinned buffer: the copy is ordered
        first, then before_readback's work is issued behind it, and only the copy is
        waited for -- that work runs under the host's line-search decision."""
        n = dev.numel()
        if self._host_buf is None or self._host_buf.numel() < n:
            self._host_buf = torch.empty(max(n, 64), dtype=torch.float64, pin_memory=True)
        h = self._host_buf[:n]
        h.copy_(dev, non_blocking=True)
        done = torch.cuda.Event()
        done.record()
        if self.before_readback is not None:
            self.before_readback()
        done.synchronize()
        return h.numpy().copy()

    # EzFlat surface (core.py:544-554)
    def get_params_flat(self):
        return self.stochpol.get_flat()

    def set_params_flat(self, th):
        self.stochpol.set_from_flat(th)

    def __call__(self, paths):
        """Per-path API (`trpo.py:72-78`): concatenate, move to device, update."""
        from .core import Batch
        batch = Batch.from_paths(paths, self.stochpol, device=self.stochpol.net.device)
        return self.update(batch)

    def update(self, batch):
        cfg, ops, comm, net = self.cfg, self.ops, self.comm, self.stochpol.net
        n_glob = batch.n_global if getattr(batch, "n_global", None) else comm.allreduce_int(batch.n)
        ops.bind(batch, 1.0 / n_glob)
        thprev = net.theta.clone()
        g, sums = ops.surrgrad()
        comm.allreduce_(g)
        comm.allreduce_(sums)
        diag = {"n_global": n_glob}
        # The conjugate gradient is issued before the host looks at g: losses_before,
        # the zero-gradient test (np.allclose(g, 0) == max|g| <= 1e-8) and the step
        # scaling come back in ONE device-to-host copy after CG, instead of a pipeline
        # drain ahead of it.  A zero gradient discards the CG result (theta untouched).
        damping, max_kl = float(cfg["cg_damping"]), float(cfg["max_kl"])
        ops.cg_init(ops.neg_g64(g))
        for _ in range(self.CG_ITERS):
            fv = ops.fvp(ops.p32, skip=ops.flag)
            comm.allreduce_(fv)
            ops.cg_update(fv, damping, self.RESIDUAL_TOL)
        step = ops.trpo_step(g, max_kl)[:4]
        # the first line-search batch (k = 0, accepted in most updates) is issued before
        # the readback and returns in the same copy: one host round trip instead of two
        # (a zero gradient discards it unread)
        first = None
        parts = [step, sums.double()[:3], g.abs().max().double().reshape(1), ops.state[:3]]
        # the rollout's abort status (a persistent launch that gave up: incomplete rows)
        # rides in the same copy, so an aborted batch never reaches theta
        abort = getattr(batch, "abort", None)
        if abort is not None:
            abort = abort.double().reshape(1)
            comm.allreduce_(abort)  # any rank's abort stops every rank
            parts.append(abort)
        if self.LS_BATCHES:
            K0 = min(self.LS_BATCHES[0], self.MAX_BACKTRACKS)
            ls_sums, ls_cand = ops.losses_batch(thprev, 0, K0)
            comm.allreduce_(ls_sums)
            parts.append(ls_sums.reshape(-1))
        host = self._readback(torch.cat(parts)) if net.theta.is_cuda else torch.cat(parts).cpu().numpy()
        if abort is not None and host[11] != 0:
            raise _lib.MrlError("policy update on an aborted rollout: " + getattr(batch, "abort_msg", ""))
        if self.LS_BATCHES:
            o = 11 + (abort is not None)
            first = (host[o:].reshape(K0, -1), ls_cand)
        losses_before = _losses(host[4:7], n_glob)
        losses_after = losses_before
        if host[7] <= 1e-8:
            print("got zero gradient. not updating")
            diag["skipped"] = True
            if self.after_theta is not None:
                self.after_theta()
        else:
            shs, lm, neggdotstepdir, rate = (float(v) for v in host[:4])
            if timing.enabled():
                skipped = self.CG_ITERS - int(host[10])  # Fisher products after convergence
                timing.drop_last("fvp_jvp_rows", skipped)
                timing.drop_last("fvp_vjp", skipped)
                timing.drop_last("fvp_onepass", skipped)
            fval = losses_before[0]
            trace = []
            if self.LS_BATCHES:
                success, frac, k, laux, accepted = self._linesearch_batched(thprev, fval, rate, n_glob, trace,
                                                                            first=first)
            else:
                def f(stepfrac):
                    l = _losses(self._candidate_losses(thprev, stepfrac), n_glob)
                    return l[0], l

                success, frac, k, laux = linesearch(f, fval, rate, max_backtracks=self.MAX_BACKTRACKS, trace=trace)
                accepted = ops.cand  # the accepted (last evaluated) candidate
            if success:
                net.theta.copy_(accepted)
                losses_after = laux
            else:
                net.theta.copy_(thprev)
            # the next rollout is issued first: it packs its own image from theta, and the
            # net's images are for this stream's next passes (off the update-to-rollout seam)
            if self.after_theta is not None:
                self.after_theta()
            net.pack()
            diag.update(skipped=False, shs=shs, lm=lm, neggdotstepdir=neggdotstepdir, expected_rate=rate,
                        success=success, k=k, stepfrac=frac, cg_iters=int(host[10]), rdotr=float(host[8]),
                        ls=np.array(trace, dtype=np.float64))
        self.last_diag = diag
        out = OrderedDict()
        for (lname, lbefore, lafter) in zip(self.loss_names, losses_before, losses_after):
            out[lname + "_before"] = lbefore
            out[lname + "_after"] = lafter
        return out

    def _linesearch_batched(self, thprev, fval, rate, n_glob, trace, accept_ratio=.1, first=None):
        """`trpo.py:143-159` with the candidates scored in batches (LS_BATCHES): each batch
        is one device call, one all-reduce of its [K, 4] sums and one readback; the
        accept test runs in the reference's order, so the first accepted k (and the
        trace up to it) equal the serial loop's.  ``first``: the first batch's (host
        sums, device candidates), already evaluated."""
        k0, bi = 0, 0
        while k0 < self.MAX_BACKTRACKS:
            # the batch sizes in order, the last one repeated until every backtrack of the
            # serial loop has been scored
            K = min(self.LS_BATCHES[min(bi, len(self.LS_BATCHES) - 1)], self.MAX_BACKTRACKS - k0)
            bi += 1
            if k0 == 0 and first is not None:
                host, cand = first
            else:
                sums, cand = self.ops.losses_batch(thprev, k0, K)
                self.comm.allreduce_(sums)
                host = sums.cpu().numpy()
            for j in range(K):
                k = k0 + j
                stepfrac = .5 ** k
                l = _losses(host[j], n_glob)
                actual = fval - l[0]
                expected = rate * stepfrac
                ratio = actual / expected
                trace.append((stepfrac, actual, expected, ratio))
                if ratio > accept_ratio and actual > 0:
                    return True, stepfrac, k, l, cand[j]
            k0 += K
        return False, None, -1, None, None

    def _candidate_losses(self, thprev, stepfrac):
        th = self.ops.candidate(thprev, stepfrac)
        sums = self.ops.losses(th)
        self.comm.allreduce_(sums)
        return sums
