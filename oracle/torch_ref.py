"""Second restatement of the Theano graph (`trpo.py:29-70`) with torch-CPU autograd
-- TEST INFRASTRUCTURE (oracle).

This follows Theano's formulation literally: ``pg = grad(surr)``, and the
Fisher-vector product as the double backward of
``kl_firstfixed = sum KL(stopgrad(p), p) / N`` (`trpo.py:45-58`).  It exists to
pin the analytic Gauss-Newton form used by ``oracle/trpo_np.py`` and by the HIP
kernels (they must agree in float64 to ~1e-15).
"""
import numpy as np
import torch


def _params(spec, theta):
    t = torch.tensor(np.asarray(theta, dtype=np.float64), requires_grad=True)
    return t


def _forward(spec, t, ob):
    x = torch.tensor(ob, dtype=torch.float64)
    i = 0
    h = x
    n_dense = len(spec.hid) + 1
    prev = spec.n_in
    for l in range(n_dense):
        out = spec.hid[l] if l < len(spec.hid) else spec.n_out
        W = t[i:i + prev * out].reshape(prev, out)
        i += prev * out
        b = t[i:i + out]
        i += out
        h = h @ W + b
        if l < n_dense - 1:
            h = torch.tanh(h)
        prev = out
    if spec.head == "softmax":
        return torch.softmax(h, dim=1)
    if spec.head == "gauss":
        logstd = t[i:i + spec.n_out]
        return torch.cat([h, torch.exp(logstd)[None, :].expand(h.shape[0], -1)], dim=1)
    return h


def _kl(spec, p0, p1):
    if spec.head == "softmax":
        return (p0 * torch.log(p0 / p1)).sum(1)
    d = spec.n_out
    m0, s0, m1, s1 = p0[:, :d], p0[:, d:], p1[:, :d], p1[:, d:]
    return torch.log(s1 / s0).sum(1) + ((s0 ** 2 + (m0 - m1) ** 2) / (2 * s1 ** 2)).sum(1) - 0.5 * d


def _loglik(spec, a, p):
    if spec.head == "softmax":
        return torch.log(p[torch.arange(p.shape[0]), torch.tensor(a, dtype=torch.long)])
    d = spec.n_out
    a = torch.tensor(a, dtype=torch.float64)
    m, s = p[:, :d], p[:, d:]
    return -0.5 * (((a - m) / s) ** 2).sum(1) - 0.5 * np.log(2 * np.pi) * d - torch.log(s).sum(1)


def fvp_double_backward(spec, theta, v, ob):
    t = _params(spec, theta)
    p = _forward(spec, t, ob)
    kl_ff = _kl(spec, p.detach(), p).sum() / ob.shape[0]
    (g,) = torch.autograd.grad(kl_ff, t, create_graph=True)
    gvp = (g * torch.tensor(np.asarray(v, dtype=np.float64))).sum()
    (fv,) = torch.autograd.grad(gvp, t)
    return fv.numpy()


def pg_autograd(spec, theta, ob, act, adv, oldprob):
    t = _params(spec, theta)
    p = _forward(spec, t, ob)
    N = ob.shape[0]
    logp = _loglik(spec, act, p)
    oldlogp = _loglik(spec, act, torch.tensor(oldprob, dtype=torch.float64))
    surr = (-1.0 / N) * (torch.exp(logp - oldlogp) * torch.tensor(adv, dtype=torch.float64)).sum()
    (g,) = torch.autograd.grad(surr, t)
    return g.numpy()
