"""PPO updaters (`ppo.py:3-229` of the reference) restated on the CPU -- TEST
INFRASTRUCTURE (oracle).

``pensurr = surr + kl_coeff * kl + cutoff_coeff * (kl > cutoff) * (kl - cutoff)^2``
(`ppo.py:46-47`, `ppo.py:153`) with kl = mean KL(old, new) (or KL(new, old) under
``reverse_kl``, `ppo.py:38-41`); its gradient is taken with torch-CPU autograd in
float64 (Theano's ``flatgrad``, `ppo.py:48`), independent of the analytic head
gradients the HIP epilogue uses.  ``lbfgs_update`` follows PpoLbfgsUpdater.__call__
(`ppo.py:59-113`), ``sgd_update`` PpoSgdUpdater.__call__ with ``adam_updates``
(`ppo.py:166-229`, `ppo.py:231-258`) for a given sequence of epoch permutations.
"""
import numpy as np
import scipy.optimize
import torch

from . import torch_ref as TR
from . import trpo_np as T


def _kl_rows(spec, p_old, p_new, reverse):
    return TR._kl(spec, p_new, p_old) if reverse else TR._kl(spec, p_old, p_new)


def losses(spec, theta, ob, act, adv, oldprob, reverse_kl=False):
    """[surr, kl, ent] (`ppo.py:50`)."""
    prob = T.policy_prob(spec, theta, ob)
    N = ob.shape[0]
    ratio = np.exp(T.loglik(spec, act, prob) - T.loglik(spec, act, oldprob))
    surr = (-1.0 / N) * ratio.dot(adv)
    kl = (T.kl(spec, prob, oldprob) if reverse_kl else T.kl(spec, oldprob, prob)).mean()
    return np.array([surr, kl, T.entropy(spec, prob).mean()])


def pensurr_and_grad(spec, theta, ob, act, adv, oldprob, kl_coeff, kl_cutoff, cutoff_coeff=1000.0,
                     reverse_kl=False, dtype=torch.float64):
    """pensurr and its autograd gradient (`ppo.py:46-48`); dtype=torch.float32 evaluates
    the graph the way Theano floatX=float32 does (inputs and parameters downcast)."""
    t = TR._params(spec, theta, dtype)
    p = TR._forward(spec, t, ob)
    N = ob.shape[0]
    logp = TR._loglik(spec, act, p)
    po = torch.tensor(np.asarray(oldprob), dtype=dtype)
    oldlogp = TR._loglik(spec, act, po)
    surr = (-1.0 / N) * (torch.exp(logp - oldlogp) * torch.tensor(np.asarray(adv), dtype=dtype)).sum()
    kl = _kl_rows(spec, po, p, reverse_kl).mean()
    pen = surr + kl_coeff * kl + cutoff_coeff * (kl > kl_cutoff).to(dtype) * (kl - kl_cutoff) ** 2
    (g,) = torch.autograd.grad(pen, t)
    return float(pen.item()), g.numpy()


def losses_t(spec, theta, ob, act, adv, oldprob, reverse_kl=False, dtype=torch.float64):
    """[surr, kl, ent] (`ppo.py:50`) on the torch graph in `dtype` (the fixtures' floatX runs)."""
    with torch.no_grad():
        t = torch.tensor(np.asarray(theta), dtype=dtype)
        p = TR._forward(spec, t, ob)
        po = torch.tensor(np.asarray(oldprob), dtype=dtype)
        N = ob.shape[0]
        surr = (-1.0 / N) * (torch.exp(TR._loglik(spec, act, p) - TR._loglik(spec, act, po))
                             * torch.tensor(np.asarray(adv), dtype=dtype)).sum()
        kl = _kl_rows(spec, po, p, reverse_kl).mean()
        if spec.head == "softmax":
            ent = (-(p * torch.log(p)).sum(1)).mean()
        else:
            d = spec.n_out
            ent = (torch.log(p[:, d:]).sum(1) + 0.5 * np.log(2 * np.pi * np.e) * d).mean()
        return [surr.numpy(), kl.numpy(), ent.numpy()]


def policy_prob_t(spec, theta, ob, dtype=torch.float64):
    with torch.no_grad():
        return TR._forward(spec, torch.tensor(np.asarray(theta), dtype=dtype), ob).numpy()


def lbfgs_update(spec, theta, ob, act, adv, oldprob, kl_coeff, kl_target=1e-2, maxiter=25, reverse_kl=False,
                 do_split=False):
    """One PpoLbfgsUpdater.__call__ (`ppo.py:59-112`): returns (theta_new, info, kl_coeff_new);
    do_split trains on the first 75 % of the rows and adds the test_* stats of the rest."""
    kl_cutoff = 2.0 * kl_target
    N = ob.shape[0]
    if do_split:
        s = int(0.75 * N)
        th, info, kc = lbfgs_update(spec, theta, ob[:s], act[:s], adv[:s], oldprob[:s], kl_coeff, kl_target, maxiter,
                                    reverse_kl)
        tb = losses(spec, theta, ob[s:], act[s:], adv[s:], oldprob[s:], reverse_kl)
        ta = losses(spec, th, ob[s:], act[s:], adv[s:], oldprob[s:], reverse_kl)
        info.update({"test_" + k: v for k, v in _info(tb, ta).items()})
        return th, info, kc

    def lossandgrad(th):
        th32 = th.astype(np.float32).astype(np.float64)  # set_params_flat casts to floatX
        l, g = pensurr_and_grad(spec, th32, ob, act, adv, oldprob, kl_coeff, kl_cutoff, reverse_kl=reverse_kl)
        return l, g.astype(np.float64)

    before = losses(spec, theta, ob, act, adv, oldprob, reverse_kl)
    th, _, _ = scipy.optimize.fmin_l_bfgs_b(lossandgrad, theta.astype(np.float64), maxiter=maxiter)
    th = th.astype(np.float32).astype(np.float64)
    after = losses(spec, th, ob, act, adv, oldprob, reverse_kl)
    kc = kl_adapt(after[1], kl_target, kl_coeff)
    return th, _info(before, after), kc


def kl_adapt(klafter, kl_target, kl_coeff):
    """`ppo.py:94-102`."""
    if klafter > 1.3 * kl_target:
        return kl_coeff * 1.5
    if klafter < 0.7 * kl_target:
        return kl_coeff / 1.5
    return kl_coeff


def _info(before, after):
    info = {}
    for name, b, a in zip(["surr", "kl", "ent"], before, after):
        info[name + "_before"] = b
        info[name + "_after"] = a
        info[name + "_change"] = a - b
    return info


def sgd_update(spec, theta, ob, act, adv, perms, kl_coeff, kl_target=1e-2, stepsize=1e-3, cutoff_coeff=1000.0,
               batchsize=128, adam_state=None, do_split=False):
    """PpoSgdUpdater.__call__ (`ppo.py:169-229`) for the given epoch permutations (over the
    training rows), float32 Adam.  do_split: the training rows are the first
    (0.75 N // batchsize) * batchsize, the test_* stats come from the rest.
    Returns (theta_new, info, kl_coeff_new, adam_state)."""
    kl_cutoff = 2.0 * kl_target
    oldprob = T.policy_prob(spec, theta, ob)          # old net = params at update start
    th = theta.astype(np.float32)
    m, v, t = adam_state if adam_state is not None else (np.zeros_like(th), np.zeros_like(th), 0)
    N = ob.shape[0]
    if do_split:
        s = (int(.75 * N) // batchsize) * batchsize
        tb = losses(spec, theta, ob[s:], act[s:], adv[s:], oldprob[s:])
        th1, info, kc, st = sgd_update(spec, theta, ob[:s], act[:s], adv[:s], perms, kl_coeff, kl_target, stepsize,
                                       cutoff_coeff, batchsize, adam_state)
        ta = losses(spec, th1, ob[s:], act[s:], adv[s:], oldprob[s:])
        info.update({"test_" + k: v for k, v in _info(tb, ta).items()})
        return th1, info, kc, st
    before = losses(spec, th.astype(np.float64), ob, act, adv, oldprob)
    b1, b2, eps = np.float32(0.9), np.float32(0.999), np.float32(1e-8)
    train_losses = before
    for perm in perms:
        mb = []
        for i in range(0, N, batchsize):
            idx = perm[i:i + batchsize]
            th64 = th.astype(np.float64)
            mb.append(losses(spec, th64, ob[idx], act[idx], adv[idx], oldprob[idx]))
            _, g = pensurr_and_grad(spec, th64, ob[idx], act[idx], adv[idx], oldprob[idx], kl_coeff, kl_cutoff,
                                    cutoff_coeff)
            g = g.astype(np.float32)
            t += 1
            a_t = np.float32(stepsize) * np.sqrt(np.float32(1) - b2 ** np.float32(t)) / (np.float32(1) - b1 ** np.float32(t))
            m = b1 * m + (np.float32(1) - b1) * g
            v = b2 * v + (np.float32(1) - b2) * g * g
            th = th - a_t * m / (np.sqrt(v) + eps)
        train_losses = np.mean(mb, axis=0)
    kc = kl_adapt(train_losses[1], kl_target, kl_coeff)
    return th.astype(np.float64), _info(before, train_losses), kc, (m, v, t)
