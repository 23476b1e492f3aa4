"""Second restatement of the Theano graph (`trpo.py:29-70`) with torch-CPU autograd
-- TEST INFRASTRUCTURE (oracle).

This follows Theano's formulation literally: ``pg = grad(surr)``, and the
Fisher-vector product as the double backward of
``kl_firstfixed = sum KL(stopgrad(p), p) / N`` (`trpo.py:45-58`).  It exists to
pin the analytic Gauss-Newton form used by ``oracle/trpo_np.py`` and by the HIP
kernels (they must agree in float64 to ~1e-15).

``dtype=torch.float32`` evaluates the same graphs the way the reference runs them
with Theano ``floatX=float32`` (`keras_theano_setup.py:5-6`): parameters, inputs and
tangent downcast to float32 (``allow_input_downcast``, ``SetFromFlat`` casts to floatX
`core.py:540`, the tangent is a ``T.fvector`` `trpo.py:48`), float32 outputs.  The VF
regression graph (`core.py:607-618`) is restated here too, for the fit fixtures.
"""
import numpy as np
import torch


F64 = torch.float64


def _params(spec, theta, dtype=F64):
    return torch.tensor(np.asarray(theta), dtype=dtype, requires_grad=True)


def _forward(spec, t, ob):
    x = torch.tensor(np.asarray(ob), dtype=t.dtype)
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
    a = torch.tensor(np.asarray(a), dtype=p.dtype)
    m, s = p[:, :d], p[:, d:]
    return -0.5 * (((a - m) / s) ** 2).sum(1) - 0.5 * np.log(2 * np.pi) * d - torch.log(s).sum(1)


def fvp_double_backward(spec, theta, v, ob, dtype=F64):
    t = _params(spec, theta, dtype)
    p = _forward(spec, t, ob)
    kl_ff = _kl(spec, p.detach(), p).sum() / ob.shape[0]
    (g,) = torch.autograd.grad(kl_ff, t, create_graph=True)
    gvp = (g * torch.tensor(np.asarray(v), dtype=dtype)).sum()
    (fv,) = torch.autograd.grad(gvp, t)
    return fv.numpy()


def pg_autograd(spec, theta, ob, act, adv, oldprob, dtype=F64):
    t = _params(spec, theta, dtype)
    p = _forward(spec, t, ob)
    N = ob.shape[0]
    logp = _loglik(spec, act, p)
    oldlogp = _loglik(spec, act, torch.tensor(np.asarray(oldprob), dtype=dtype))
    surr = (-1.0 / N) * (torch.exp(logp - oldlogp) * torch.tensor(np.asarray(adv), dtype=dtype)).sum()
    (g,) = torch.autograd.grad(surr, t)
    return g.numpy()


def losses(spec, theta, ob, act, adv, oldprob, dtype=F64):
    """[surr, mean KL(old, new), mean entropy] (`trpo.py:42,60-64`)."""
    with torch.no_grad():
        t = torch.tensor(np.asarray(theta), dtype=dtype)
        p = _forward(spec, t, ob)
        N = ob.shape[0]
        old = torch.tensor(np.asarray(oldprob), dtype=dtype)
        surr = (-1.0 / N) * (torch.exp(_loglik(spec, act, p) - _loglik(spec, act, old))
                             * torch.tensor(np.asarray(adv), dtype=dtype)).sum()
        kl = _kl(spec, old, p).mean()
        if spec.head == "softmax":
            ent = (-(p * torch.log(p)).sum(1)).mean()
        else:
            d = spec.n_out
            ent = (torch.log(p[:, d:]).sum(1) + 0.5 * np.log(2 * np.pi * np.e) * d).mean()
        return [surr.numpy(), kl.numpy(), ent.numpy()]


# ------------------------------------------------ VF regression graph (core.py:607-618)
VF_L2 = 1e-3


def _vf_terms(spec, t, X, ytarg):
    ypred = _forward(spec, t, X)
    y = torch.tensor(np.asarray(ytarg), dtype=t.dtype).reshape(ypred.shape)
    N = X.shape[0]
    mse = torch.square(y - ypred).sum() / N
    l2 = VF_L2 * torch.square(t).sum()  # every trainable weight, biases included (core.py:613)
    return mse + l2, mse, l2


def vf_predict(spec, theta, X, dtype=F64):
    with torch.no_grad():
        return _forward(spec, torch.tensor(np.asarray(theta), dtype=dtype), X).numpy()


def vf_lossgrad(spec, theta, X, ytarg, dtype=F64):
    """``f_lossgrad`` (`core.py:670`): [loss, flatgrad(loss)]."""
    t = _params(spec, theta, dtype)
    loss, _, _ = _vf_terms(spec, t, X, ytarg)
    (g,) = torch.autograd.grad(loss, t)
    return loss.detach().numpy(), g.numpy()


def vf_losses(spec, theta, X, ytarg, dtype=F64):
    """``f_losses`` (`core.py:671`): [loss, mse, l2]."""
    with torch.no_grad():
        return [v.numpy() for v in _vf_terms(spec, torch.tensor(np.asarray(theta), dtype=dtype), X, ytarg)]
