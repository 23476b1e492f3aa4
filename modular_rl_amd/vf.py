"""Value-function baseline on device (`core.py:595-697` of the reference).

``NnVf`` / ``NnRegression`` / ``LbfgsOptimizer`` keep the reference's names and
semantics: the VF input is ``[obs, t / timestep_limit]`` (`core.py:659-660`), the
regression target is ``mixfrac * return + (1 - mixfrac) * V_old`` (`core.py:622-
624`), and the loss ``sum((y - yhat)^2)/N + 1e-3 * sum(theta^2)`` (`core.py:611-617`)
is minimised by scipy's L-BFGS-B for ``maxiter`` iterations (`core.py:686-687`) on
the host, while every loss+gradient evaluation is one fused forward pass
(``mrl_mlp_rows`` VFLOSS) + one VJP (``mrl_mlp_vjp``) on the GPU, all-reduced over
ranks in data-parallel mode.
"""
import contextlib
from collections import OrderedDict

import numpy as np
import scipy.optimize
import torch

from . import _lib, timing
from ._lib import call, ptr, stream
from .dist import Comm

L2_COEF = 1e-3


class DeviceMoments:
    """numpy std of (a - b) over all rows of all ranks, as numpy computes it: two
    passes (the global mean, then the sums of the centred values), one host read."""

    def __init__(self, device, comm):
        self.device, self.comm = device, comm
        self.out = torch.zeros(2, 3, dtype=torch.float64, device=device)
        self.ws = None

    def std(self, a, b, n):
        nbytes = int(_lib.load().mrl_moments_workspace_bytes(int(n)))
        if self.ws is None or self.ws.numel() * 8 < nbytes:
            self.ws = torch.empty(nbytes // 8 + 1, dtype=torch.float64, device=self.device)
        call("mrl_moments", ptr(a), ptr(b), int(n), ptr(self.out[0]), ptr(self.ws), stream())
        self.comm.allreduce_(self.out[0])
        call("mrl_moments_centered", ptr(a), ptr(b), int(n), ptr(self.out[0]), ptr(self.out[1]), ptr(self.ws),
             stream())
        self.comm.allreduce_(self.out[1])
        s, s2, c = (float(v) for v in self.out[1].cpu().numpy())
        d = s / c
        return float(np.sqrt(max(s2 / c - d * d, 0.0)))


class LbfgsOptimizer:
    """scipy L-BFGS-B driver; loss and gradient evaluated on device (`core.py:663-697`)."""

    def __init__(self, net, maxiter=3, comm=None):
        self.net = net
        self.maxiter = maxiter
        self.comm = comm if comm is not None else Comm()
        self.g = torch.zeros(net.P, dtype=torch.float32, device=net.device)
        self.sums = torch.zeros(4, dtype=torch.float64, device=net.device)
        self.n_evals = 0

    def get_params_flat(self):
        return self.net.get_flat()

    def set_params_flat(self, th):
        self.net.set_flat(th)

    def _eval(self, data, with_grad):
        net = self.net
        x, ep_t, limit, n, target, n_glob = data
        ghead = net.ws.get("vf_ghead", n, torch.float32)
        partial = net.ws.get("vf_partial", net.partial_rows(n) * 4, torch.float64)
        net.rows(_lib.EPI_VFLOSS, x, n, ep_t=ep_t, timestep_limit=limit, inv_n_global=1.0 / n_glob, target=target,
                 ghead=ghead, partial=partial)
        net.reduce_partial(partial, n, self.sums)
        if with_grad:
            timing.start("vf_vjp", detail=True)
            net.vjp_flat(x, n, ghead, self.g, ep_t=ep_t, timestep_limit=limit)
            timing.stop("vf_vjp")
            self.comm.allreduce_(self.g)
        self.comm.allreduce_(self.sums)
        th = net.theta.detach().double().cpu().numpy()
        mse = float(self.sums[0].item()) / n_glob
        l2 = L2_COEF * float(np.sum(th * th))
        g = None
        if with_grad:
            g = self.g.detach().double().cpu().numpy() + 2.0 * L2_COEF * th
        return mse + l2, mse, l2, g

    def update(self, data):
        thprev = self.get_params_flat()
        memo = {}  # float32 theta bytes -> (loss, mse, l2, grad): scipy revisits points

        def evaluate(th32, with_grad):
            key = th32.tobytes()
            hit = memo.get(key)
            if hit is not None and (hit[3] is not None or not with_grad):
                return hit
            if not np.array_equal(th32, self.net.theta.detach().cpu().numpy()):
                self.set_params_flat(th32)
            self.n_evals += 1
            r = self._eval(data, with_grad)
            memo[key] = r
            return r

        def lossandgrad(th):
            l, _, _, g = evaluate(th.astype(np.float32), True)
            return l, g.astype("float64")

        x, ep_t, n = data[0], data[1], data[3]
        pin = getattr(self.net, "pin_input", None)  # the fit's rows are fixed: build the tape input once
        with (pin(x, n, ep_t) if pin is not None else contextlib.nullcontext()):
            lb, mb, l2b, _ = evaluate(thprev.astype(np.float32), True)  # scipy's first point is thprev
            theta, _, opt_info = scipy.optimize.fmin_l_bfgs_b(lossandgrad, thprev.astype(np.float64),
                                                              maxiter=self.maxiter)
            la, ma, l2a, _ = evaluate(theta.astype(np.float32), False)
        self.set_params_flat(theta)
        info = OrderedDict()
        for name, b, a in (("loss", lb, la), ("mse", mb, ma), ("l2", l2b, l2a)):
            info[name + "_before"] = b
            info[name + "_after"] = a
        self.last_opt_info = {k: v for k, v in opt_info.items() if k != "grad"}
        return info


class NnRegression:
    """`core.py:595-637`: mixfrac target, L-BFGS fit, prediction / EV statistics."""

    def __init__(self, net, mixfrac=1.0, maxiter=2, comm=None):
        self.net = net
        self.mixfrac = mixfrac
        self.comm = comm if comm is not None else Comm()
        self.opt = LbfgsOptimizer(net, maxiter=maxiter, comm=self.comm)
        self.moments = DeviceMoments(net.device, self.comm)

    def set_comm(self, comm):
        """Rebind every collective of the fit (loss / gradient sums, row count, the VF
        statistics' moments) to `comm` -- e.g. Comm.host() while the fit overlaps the
        rollout in data-parallel mode."""
        self.comm = comm
        self.opt.comm = comm
        self.moments.comm = comm

    def predict(self, x, n, ep_t=None, timestep_limit=1.0, out=None, feat_out=None):
        return self.net.forward(x, n, ep_t=ep_t, timestep_limit=timestep_limit, out=out, feat_out=feat_out)

    def fit(self, x, n, ytarg, ep_t=None, timestep_limit=1.0, ypredold=None, n_global=None):
        """ytarg: [n] device returns. ypredold: V_old predictions if already computed
        (compute_advantage evaluates the same net on the same rows, core.py:70)."""
        net = self.net
        if ypredold is None:
            ypredold = self.predict(x, n, ep_t, timestep_limit)
        target = net.ws.get("vf_target", n, torch.float32)
        call("mrl_vf_target", ptr(ytarg), ptr(ypredold), float(self.mixfrac), int(n), ptr(target), stream())
        n_glob = n_global if n_global else self.comm.allreduce_int(n)
        out = self.opt.update((x, ep_t, timestep_limit, n, target, n_glob))
        yprednew = self.predict(x, n, ep_t, timestep_limit, out=net.ws.get("vf_pred_new", n, torch.float32))
        out["PredStdevBefore"] = self.moments.std(ypredold, None, n)
        out["PredStdevAfter"] = self.moments.std(yprednew, None, n)
        vary = self.moments.std(ytarg, None, n) ** 2
        out["TargStdev"] = float(np.sqrt(vary))

        def ev(yp):  # explained_variance_2d (misc_utils.py:44-49)
            if vary < 1e-10:
                return 0.0
            return 1.0 - self.moments.std(ytarg, yp, n) ** 2 / vary

        out["EV_before"] = ev(ypredold)
        out["EV_after"] = ev(yprednew)
        return out


class NnVf:
    """Value baseline with the time feature (`core.py:643-660`)."""

    def __init__(self, net, timestep_limit, regression_params, comm=None):
        self.reg = NnRegression(net, comm=comm, **regression_params)
        self.timestep_limit = timestep_limit
        self._feat_gen = 0

    @property
    def net(self):
        return self.reg.net

    def preproc(self, ob_no):
        return np.concatenate([ob_no, np.arange(len(ob_no)).reshape(-1, 1) / float(self.timestep_limit)], axis=1)

    def predict(self, path):
        ob = torch.as_tensor(np.asarray(path["observation"], dtype=np.float32)).to(self.net.device)
        n = ob.shape[0]
        ep_t = torch.arange(n, dtype=torch.int32, device=self.net.device)
        return self.reg.predict(ob, n, ep_t, self.timestep_limit).cpu().numpy().astype(np.float64)

    def _features_buf(self, n):
        self._feat_gen += 1
        return self.net.ws.get("vf_features", int(n) * self.net.n_in, torch.float32)

    def features(self, obs, n, ep_t):
        """X = [obs, t / timestep_limit] materialised once per batch (`core.py:659-660`):
        every VF pass of the fit then reads plain rows instead of re-deriving the time
        feature per tile."""
        n = int(n)
        X = self._features_buf(n)
        call("mrl_concat_time", ptr(obs), ptr(ep_t), n, self.net.n_in - 1, float(self.timestep_limit), ptr(X), 0,
             stream())
        return X

    def predict_batch(self, batch, out=None):
        """V_old of the batch (`core.py:70`) straight from the rollout's rows, the time
        feature derived per row; the same pass writes the rows it derived, [obs, t /
        limit], as the fit's materialised features (``feat_out``: no separate copy, all
        on the caller's stream, so nothing reads the rollout's rows after this returns)."""
        X = self._features_buf(batch.n)
        y = self.reg.predict(batch.obs, batch.n, batch.ep_t, self.timestep_limit, out=out, feat_out=X)
        # the fit of this batch reuses the features while no other batch's have replaced them
        batch.vf_x = (X, self._feat_gen)
        return y

    def fit_batch(self, batch):
        cached = getattr(batch, "vf_x", None)
        if cached is not None and cached[1] == self._feat_gen:
            X = cached[0]
        else:
            # the features must come from this batch's own rows: once the next rollout is
            # issued into the same buffers (the pipelined loop), they are another iteration's
            if hasattr(batch, "rows_valid") and not batch.rows_valid():
                raise _lib.MrlError("NnVf.fit_batch: the batch's VF features were replaced and its rows already "
                               "hold the next rollout; predict_batch must be the last VF pass before the fit")
            X = self.features(batch.obs, batch.n, batch.ep_t)
        return self.reg.fit(X, batch.n, batch.ret, None, 1.0, ypredold=batch.vpred,
                            n_global=getattr(batch, "n_global", None))

    def fit(self, paths):
        from .core import Batch
        batch = Batch.from_paths(paths, None, device=self.net.device, need_policy=False)
        batch.ret = torch.as_tensor(np.concatenate([p["return"] for p in paths]).astype(np.float32)).to(self.net.device)
        batch.vpred = None
        return self.reg.fit(batch.obs, batch.n, batch.ret, batch.ep_t, self.timestep_limit)
