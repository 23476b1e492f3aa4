"""Oracle-backed stand-in for modular_rl_amd.trpo.HipTrpoOps -- TEST ONLY.

Lets the real TrpoUpdater.update orchestration (collective placement, global-N
scaling, CG control flow, line search) run on CPU under gloo: every device
kernel the updater calls is replaced by the float64 numpy oracle on this rank's
local rows, returning LOCAL sums scaled by 1/N_global exactly like the kernels.
"""
import types

import numpy as np
import torch

from oracle import trpo_np as T


def fake_policy(spec, theta):
    net = types.SimpleNamespace(theta=torch.tensor(theta, dtype=torch.float64), pack=lambda *a, **k: None,
                                device=torch.device("cpu"), P=spec.P)
    return types.SimpleNamespace(net=net, get_flat=lambda: net.theta.numpy().copy(),
                                 set_from_flat=lambda th: net.theta.copy_(torch.as_tensor(th)))


class OracleOps:
    def __init__(self, spec, net):
        self.spec, self.net, self.P = spec, net, spec.P
        z = lambda: torch.zeros(self.P, dtype=torch.float64)  # noqa: E731
        self.x, self.r, self.p, self.p32, self.fullstep, self.cand, self.ax = z(), z(), z(), z(), z(), z(), z()
        self.state = torch.zeros(4, dtype=torch.float64)
        self.flag = torch.zeros(2, dtype=torch.int32)
        self.fv = z()

    def bind(self, batch, inv_ng):
        self.b, self.inv_ng = batch, inv_ng

    def _scale(self):
        return self.b.n * self.inv_ng  # oracle divides by local n; kernels by N_global

    def surrgrad(self):
        b, th = self.b, self.net.theta.numpy()
        g = T.policy_gradient(self.spec, th, b.obs, b.act, b.adv, b.prob) * self._scale()
        return torch.tensor(g), self.losses(self.net.theta)

    def losses(self, theta):
        b = self.b
        s, kl, ent = T.surr_kl_ent(self.spec, theta.numpy(), b.obs, b.act, b.adv, b.prob)
        return torch.tensor([-s * b.n, kl * b.n, ent * b.n, 0.0])

    def fvp(self, v, skip=None):
        if skip is not None and int(skip[0]) != 0:
            return self.fv
        fv = T.fisher_vector_product(self.spec, self.net.theta.numpy(), v.numpy(), self.b.obs) * self._scale()
        self.fv = torch.tensor(fv)
        return self.fv

    def neg_g64(self, g):
        return -g.double()

    def cg_init(self, b):
        self.x.zero_()
        self.ax.zero_()
        self.r.copy_(b)
        self.p.copy_(b)
        self.p32.copy_(b)
        self.state[0] = float(b.dot(b))
        self.state[2] = 0
        self.flag[0] = 0

    def cg_update(self, fv, damping, tol):
        if int(self.flag[0]) != 0:
            return
        rdotr = float(self.state[0])
        z = fv + damping * self.p
        v = np.float64(rdotr) / np.float64(self.p.dot(z))  # 0 / 0 = NaN like the device (zero gradient)
        self.x += v * self.p
        self.ax += v * z
        self.r -= v * z
        newr = float(self.r.dot(self.r))
        self.p.copy_(self.r + float(np.float64(newr) / np.float64(rdotr)) * self.p)
        self.p32.copy_(self.p)
        self.state[0] = newr
        self.state[2] += 1
        if newr < tol:
            self.flag[0] = 1

    def trpo_step(self, g, max_kl):
        shs = 0.5 * float(self.x.dot(self.ax))
        lm = np.sqrt(shs / max_kl)
        self.fullstep.copy_(self.x / lm)
        ngx = -float(g.double().dot(self.x))
        return torch.tensor([shs, lm, ngx, ngx / lm])

    def candidate(self, theta_old, frac):
        self.cand.copy_(theta_old + frac * self.fullstep)
        return self.cand

    def losses_batch(self, theta_old, k0, K):
        """Stand-in for HipTrpoOps.losses_batch: [K, 4] sums of theta_old + .5^(k0+k) fullstep."""
        cand = torch.stack([theta_old + (.5 ** (k0 + k)) * self.fullstep for k in range(K)])
        return torch.stack([self.losses(c) for c in cand]), cand


class OracleVfNet:
    """Oracle-backed stand-in for the value-function MlpNet under vf.LbfgsOptimizer --
    TEST ONLY.  rows(EPI_VFLOSS) returns this rank's squared-error sum and the head
    gradient rows 2 (v - y) / N_global like the kernel; vjp_flat backpropagates them
    through the float64 oracle.  theta holds float32 values, as on the device."""

    def __init__(self, spec, theta):
        self.spec, self.P, self.device = spec, spec.P, torch.device("cpu")
        self.theta = torch.tensor(np.asarray(theta, np.float32), dtype=torch.float64)
        self.ws = types.SimpleNamespace(get=lambda name, n, dtype: torch.zeros(n, dtype=torch.float64))
        self._acts = None

    def get_flat(self):
        return self.theta.numpy().astype(np.float32)

    def set_flat(self, th):
        self.theta.copy_(torch.as_tensor(np.asarray(th, np.float32), dtype=torch.float64))

    def partial_rows(self, n):
        return 1

    def rows(self, epi, x, n, ep_t=None, timestep_limit=1.0, inv_n_global=1.0, target=None, ghead=None,
             partial=None):
        z, self._acts = T.mlp_forward(self.spec, self.theta.numpy(), x)
        err = z[:, 0] - target.numpy()
        partial.zero_()
        partial[0] = float(np.sum(err * err))
        ghead.copy_(torch.as_tensor(2.0 * err * inv_n_global))

    def reduce_partial(self, partial, n, sums):
        sums.copy_(partial[:4])
        return sums

    def vjp_flat(self, x, n, ghead, g, ep_t=None, timestep_limit=1.0):
        gz = ghead.numpy().reshape(-1, 1)
        g.copy_(torch.as_tensor(T.flatten(T.mlp_vjp(self.spec, self.theta.numpy(), self._acts, gz))))
