"""PPO updaters (`ppo.py:3-229` of the reference) on the same device kernels as TRPO.

Both keep the reference constructor, ``options``, ``kl_coeff`` adaptation
(`ppo.py:94-102`) and the ``surr/kl/ent _before/_after/_change`` info dict.

``PpoLbfgsUpdater`` minimises ``pensurr = surr + kl_coeff kl + 1000 (kl > 2 kl_target)
(kl - 2 kl_target)^2`` with scipy's L-BFGS on the host (as the reference); each
loss/grad evaluation is one fused pass with the PPOGRAD epilogue (head gradient of
surr + c * kl, c = d pensurr / d kl) plus one VJP on the device.  c depends on the
batch KL at theta: the pass is run with the optimistic c = kl_coeff and re-run
only when the KL lands beyond the cutoff.

``PpoSgdUpdater`` runs ``epochs`` passes of 128-row minibatch Adam (`ppo.py:166-229`):
per minibatch one PPOSGD launch (forward, block-reduced minibatch KL, pensurr head
gradient), one VJP and one fused Adam step (``mrl_adam_step``); the epoch
permutation (host ``np.random.permutation``, as the reference) gathers the rows on
the device (``mrl_gather_rows``).

Data-parallel: PpoLbfgs all-reduces the loss sums and gradient of every
evaluation (all ranks take identical L-BFGS steps); PpoSgd averages each
minibatch gradient over ranks (each rank draws its own minibatches).
"""
from collections import OrderedDict

import numpy as np
import scipy.optimize
import torch

from . import _lib
from ._lib import call, ptr, stream
from .dist import Comm
from .misc_utils import update_default_config

LOSS_NAMES = ["surr", "kl", "ent"]


def _info(before, after, prefix=""):
    info = OrderedDict()
    for name, b, a in zip(LOSS_NAMES, before, after):
        info[prefix + name + "_before"] = float(b)
        info[prefix + name + "_after"] = float(a)
        info[prefix + name + "_change"] = float(a - b)
    return info


def _kl_adapt(upd, klafter):
    kt = upd.cfg["kl_target"]
    if klafter > 1.3 * kt:
        upd.kl_coeff *= 1.5
        print("Got KL=%.3f (target %.3f). Increasing penalty coeff => %.3f." % (klafter, kt, upd.kl_coeff))
    elif klafter < 0.7 * kt:
        upd.kl_coeff /= 1.5
        print("Got KL=%.3f (target %.3f). Decreasing penalty coeff => %.3f." % (klafter, kt, upd.kl_coeff))
    else:
        print("KL=%.3f is close enough to target %.3f." % (klafter, kt))


class _Rows:
    """A contiguous row range of a device batch."""

    def __init__(self, batch, lo, hi):
        self.n = int(hi - lo)
        self.obs = batch.obs[lo:hi]
        self.act = batch.act[lo:hi]
        self.adv = batch.adv[lo:hi]
        self.prob = batch.prob[lo:hi]


class _PpoBase:
    def __init__(self, stochpol, usercfg, comm):
        self.cfg = update_default_config(self.options, usercfg)
        self.stochpol = stochpol
        self.comm = comm if comm is not None else Comm()
        self.kl_coeff = 1.0
        self.loss_names = list(LOSS_NAMES)
        net = stochpol.net
        dev = net.device
        self.g = torch.zeros(net.P, dtype=torch.float32, device=dev)
        self.sums = torch.zeros(4, dtype=torch.float64, device=dev)

    def get_params_flat(self):
        return self.stochpol.get_flat()

    def set_params_flat(self, th):
        self.stochpol.set_from_flat(th)

    # updater state for checkpoints (the reference pickles the whole agent)
    def state_arrays(self):
        return {"kl_coeff": np.array([self.kl_coeff], dtype=np.float64)}

    def load_state_arrays(self, st):
        self.kl_coeff = float(np.asarray(st["kl_coeff"]).reshape(-1)[0])

    def __call__(self, paths):
        from .core import Batch
        batch = Batch.from_paths(paths, self.stochpol, device=self.stochpol.net.device)
        return self.update(batch)

    def _losses(self, rows, n_glob, epi=_lib.EPI_LOSSES, ghead=None, kl_coeff=0.0, reverse_kl=0, theta=None):
        net = self.stochpol.net
        partial = net.ws.get("ppo_partial", net.partial_rows(rows.n) * 4, torch.float64)
        net.rows(epi, rows.obs, rows.n, inv_n_global=1.0 / n_glob, act=rows.act, adv=rows.adv, oldprob=rows.prob,
                 ghead=ghead, partial=partial, theta=theta, kl_coeff=kl_coeff, reverse_kl=reverse_kl)
        net.reduce_partial(partial, rows.n, self.sums)
        self.comm.allreduce_(self.sums)
        s = self.sums.cpu().numpy()
        return np.array([-s[0] / n_glob, s[1] / n_glob, s[2] / n_glob])


class PpoLbfgsUpdater(_PpoBase):
    options = [
        ("kl_target", float, 1e-2, "Desired KL divergence between old and new policy"),
        ("maxiter", int, 25, "Maximum number of iterations"),
        ("reverse_kl", int, 0, "kl[new, old] instead of kl[old, new]"),
        ("do_split", int, 0, "Do train/test split on batches"),
    ]
    CUTOFF_COEFF = 1000.0

    def __init__(self, stochpol, usercfg, comm=None):
        super().__init__(stochpol, usercfg, comm)
        self.last_opt_info = None

    def update(self, batch):
        cfg, net, comm = self.cfg, self.stochpol.net, self.comm
        if hasattr(batch, "check_abort"):
            batch.check_abort(comm)  # an aborted persistent rollout never reaches theta
        N = batch.n
        train_stop = int(0.75 * N) if cfg["do_split"] else N
        train = _Rows(batch, 0, train_stop)
        n_glob = comm.allreduce_int(train.n)
        rev = int(cfg["reverse_kl"])
        cutoff = 2.0 * cfg["kl_target"]
        ghead = net.ws.get("ppo_ghead", train.n * net.gh, torch.float32)
        th_dev = torch.zeros(net.P, dtype=torch.float32, device=net.device)
        evals = [0]

        def lossandgrad(th):
            evals[0] += 1
            th_dev.copy_(torch.as_tensor(th, dtype=torch.float32))  # SetFromFlat casts to floatX
            net.theta.copy_(th_dev)
            net.pack()
            c = self.kl_coeff
            l = self._losses(train, n_glob, _lib.EPI_PPOGRAD, ghead, c, rev)
            kl = l[1]
            if kl > cutoff:  # penalty slope d pensurr / d kl at this theta
                c = self.kl_coeff + 2.0 * self.CUTOFF_COEFF * (kl - cutoff)
                l = self._losses(train, n_glob, _lib.EPI_PPOGRAD, ghead, c, rev)
            net.vjp_flat(train.obs, train.n, ghead, self.g)
            comm.allreduce_(self.g)
            pen = l[0] + self.kl_coeff * kl + self.CUTOFF_COEFF * float(kl > cutoff) * (kl - cutoff) ** 2
            return pen, self.g.double().cpu().numpy()

        thprev = net.theta.detach().double().cpu().numpy()
        before = self._losses(train, n_glob, reverse_kl=rev)
        test = None
        if cfg["do_split"]:
            test = _Rows(batch, train_stop, N)
            n_test = comm.allreduce_int(test.n)
            test_before = self._losses(test, n_test, reverse_kl=rev)
        theta, _, opt_info = scipy.optimize.fmin_l_bfgs_b(lossandgrad, thprev, maxiter=cfg["maxiter"])
        del opt_info["grad"]
        opt_info["evals"] = evals[0]
        self.last_opt_info = opt_info
        print(opt_info)
        self.set_params_flat(theta)
        after = self._losses(train, n_glob, reverse_kl=rev)
        _kl_adapt(self, after[1])
        info = _info(before, after)
        if test is not None:
            info.update(_info(test_before, self._losses(test, n_test, reverse_kl=rev), "test_"))
        return info


class PpoSgdUpdater(_PpoBase):
    options = [
        ("kl_target", float, 1e-2, ""),
        ("epochs", int, 10, ""),
        ("stepsize", float, 1e-3, ""),
        ("do_split", int, 0, "do train/test split"),
        ("kl_cutoff_coeff", float, 1000.0, ""),
    ]
    BATCHSIZE = _lib.PPO_BLOCK_ROWS
    BETA1, BETA2, EPS = 0.9, 0.999, 1e-8

    def __init__(self, stochpol, usercfg, comm=None):
        super().__init__(stochpol, usercfg, comm)
        net = stochpol.net
        self.m = torch.zeros(net.P, dtype=torch.float32, device=net.device)
        self.v = torch.zeros(net.P, dtype=torch.float32, device=net.device)
        self.t = 0

    def state_arrays(self):
        st = super().state_arrays()
        st.update(adam_m=self.m, adam_v=self.v, adam_t=np.array([self.t], dtype=np.int64))
        return st

    def load_state_arrays(self, st):
        super().load_state_arrays(st)
        for name, dst in (("adam_m", self.m), ("adam_v", self.v)):
            src = torch.as_tensor(np.asarray(st[name]), dtype=torch.float32)
            if src.numel() != dst.numel():
                raise ValueError(f"snapshot {name} has {src.numel()} entries, the policy has {dst.numel()}")
            dst.copy_(src.to(dst.device))
        self.t = int(np.asarray(st["adam_t"]).reshape(-1)[0])

    def _a_t(self):
        """a_t = lr sqrt(1 - b2^t) / (1 - b1^t) in floatX (`ppo.py:240`)."""
        f = np.float32
        t = f(self.t)
        return float(f(self.cfg["stepsize"]) * np.sqrt(f(1) - f(self.BETA2) ** t) / (f(1) - f(self.BETA1) ** t))

    def update(self, batch):
        cfg, net, comm = self.cfg, self.stochpol.net, self.comm
        if hasattr(batch, "check_abort"):
            batch.check_abort(comm)  # an aborted persistent rollout never reaches theta
        N, bs = batch.n, self.BATCHSIZE
        # the old network = the parameters at the start of the update (update_old_net, ppo.py:171)
        oldprob = net.forward(batch.obs, N).reshape(N, -1)
        full = _Rows(batch, 0, N)
        full.prob = oldprob
        if cfg["do_split"]:
            train_stop = (int(.75 * N) // bs) * bs
            test = _Rows(batch, train_stop, N)
            test.prob = oldprob[train_stop:]
            n_test = comm.allreduce_int(test.n)
            test_before = self._losses(test, n_test)
        else:
            train_stop = N
        train = _Rows(batch, 0, train_stop)
        train.prob = oldprob[:train_stop]
        before = self._losses(train, comm.allreduce_int(train_stop))
        dev = net.device
        pobs = torch.empty_like(train.obs)
        pact = torch.empty_like(train.act)
        padv = torch.empty_like(train.adv)
        pold = torch.empty_like(train.prob)
        ghead = net.ws.get("ppo_ghead", bs * net.gh, torch.float32)
        nmb = (train_stop + bs - 1) // bs
        mb_partial = torch.zeros(nmb, 4, 4, dtype=torch.float64, device=dev)
        mb_n = np.array([min(bs, train_stop - i) for i in range(0, train_stop, bs)], dtype=np.float64)
        train_losses = before
        s = stream()
        for _ in range(cfg["epochs"]):
            perm = torch.as_tensor(np.random.permutation(train_stop).astype(np.int64)).to(dev)
            for src, dst in ((train.obs, pobs), (train.act, pact), (train.adv, padv), (train.prob, pold)):
                call("mrl_gather_rows", ptr(src), ptr(perm), train_stop, src[0].numel() * src.element_size(),
                     ptr(dst), s)
            for k, i in enumerate(range(0, train_stop, bs)):
                n = int(mb_n[k])
                net.rows(_lib.EPI_PPOSGD, pobs[i:i + n], n, inv_n_global=1.0 / n, act=pact[i:i + n],
                         adv=padv[i:i + n], oldprob=pold[i:i + n], ghead=ghead, partial=mb_partial[k],
                         kl_coeff=self.kl_coeff, kl_cutoff=2.0 * cfg["kl_target"],
                         cutoff_coeff=cfg["kl_cutoff_coeff"])
                net.vjp_flat(pobs[i:i + n], n, ghead, self.g)
                if comm.enabled and comm.world > 1:
                    comm.allreduce_(self.g)
                    self.g.mul_(1.0 / comm.world)
                self.t += 1
                call("mrl_adam_step", ptr(net.theta), ptr(self.g), ptr(self.m), ptr(self.v), self._a_t(), self.BETA1,
                     self.BETA2, self.EPS, net.P, s)
                net.pack()
            sums = mb_partial.sum(dim=1).cpu().numpy()  # [nmb, 4]
            mb_losses = np.stack([-sums[:, 0] / mb_n, sums[:, 1] / mb_n, sums[:, 2] / mb_n], axis=1)
            train_losses = mb_losses.mean(axis=0)
            if comm.enabled and comm.world > 1:
                tl = torch.as_tensor(train_losses, dtype=torch.float64, device=dev)
                comm.allreduce_(tl)
                train_losses = tl.cpu().numpy() / comm.world
        _kl_adapt(self, train_losses[1])
        info = _info(before, train_losses)
        if cfg["do_split"]:
            info.update(_info(test_before, self._losses(test, n_test), "test_"))
        return info
