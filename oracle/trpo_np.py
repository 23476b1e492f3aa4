"""numpy restatement of the reference TRPO hot path -- TEST INFRASTRUCTURE (oracle).

Default dtype float64 ("truth").  Passing ``dtype=np.float32`` mimics the
reference's floatX=float32 Theano graph (`keras_theano_setup.py:5-9`):
parameters, activations and per-row math in float32, CG/linesearch in float64.

Flat parameter layout (`core.py:518-557`, Keras ``trainable_weights`` order,
`agentzoo.py:34-48`): [W1 (in,out) row-major, b1, ..., WL, bL, (logstd)].
"""
from collections import OrderedDict

import numpy as np
import scipy.optimize

LOG2PI = np.log(2.0 * np.pi)


# ============================================================== math utils
def discount(x, gamma):
    """y[t] = x[t] + gamma*y[t+1] (`misc_utils.py:9-27`, loop form of `a.py:15-23`)."""
    x = np.asarray(x)
    y = np.zeros_like(x, dtype=np.float64)
    v = 0.0
    for t in reversed(range(len(x))):
        v = v * gamma + x[t]
        y[t] = v
    return y


def explained_variance(ypred, y):
    """`misc_utils.py:29-42`."""
    vary = np.var(y)
    return np.nan if vary == 0 else 1 - np.var(y - ypred) / vary


def explained_variance_2d(ypred, y):
    """`misc_utils.py:44-49`."""
    vary = np.var(y, axis=0)
    out = 1 - np.var(y - ypred) / vary
    out[vary < 1e-10] = 0
    return out


# ============================================================== filters
class RunningStat:
    """Welford running moments (`running_stat.py:4-33`)."""

    def __init__(self, shape):
        self.n = 0
        self.M = np.zeros(shape)
        self.S = np.zeros(shape)

    def push(self, x):
        x = np.asarray(x)
        self.n += 1
        if self.n == 1:
            self.M[...] = x
        else:
            old = self.M.copy()
            self.M[...] = old + (x - old) / self.n
            self.S[...] = self.S + (x - old) * (x - self.M)

    def push_batch(self, xs):
        """Merge a batch of B samples in one Chan step (batched-collector
        semantics).  For B == 1 it is operation-for-
        operation the sequential ``push`` above."""
        xs = np.asarray(xs, dtype=np.float64)
        nb = xs.shape[0]
        if nb == 0:
            return
        mb = xs.mean(axis=0) if nb > 1 else xs[0].copy()
        m2b = ((xs - mb) ** 2).sum(axis=0) if nb > 1 else np.zeros_like(mb)
        self.merge(nb, mb, m2b)

    def merge(self, nb, mb, m2b):
        na = self.n
        n = na + nb
        delta = mb - self.M
        newM = self.M + (delta * nb) / n
        self.S = self.S + m2b + delta * (mb - newM) * nb
        self.M = newM
        self.n = n

    @property
    def var(self):
        return self.S / (self.n - 1) if self.n > 1 else np.square(self.M)

    @property
    def std(self):
        return np.sqrt(self.var)


class ZFilter:
    """y = clip((x - mean) / (std + 1e-8), +-clip) with a stat push first (`filters.py:17-40`)."""

    def __init__(self, shape, demean=True, destd=True, clip=10.0):
        self.demean, self.destd, self.clip = demean, destd, clip
        self.rs = RunningStat(shape)

    def __call__(self, x, update=True):
        if update:
            self.rs.push(x)
        return self.apply(x)

    def apply(self, x):
        if self.demean:
            x = x - self.rs.M
        if self.destd:
            x = x / (self.rs.std + 1e-8)
        if self.clip:
            x = np.clip(x, -self.clip, self.clip)
        return x


# ============================================================== parameters
def mlp_shapes(n_in, hid, n_out, gauss):
    """Keras Dense stack (`agentzoo.py:25-60`) + ConcatFixedStd logstd (`core.py:708-725`)."""
    shapes = []
    prev = n_in
    for h in hid:
        shapes += [(prev, h), (h,)]
        prev = h
    shapes += [(prev, n_out), (n_out,)]
    if gauss:
        shapes += [(n_out,)]
    return shapes


def n_params(shapes):
    return int(sum(np.prod(s) for s in shapes))


def unflatten(theta, shapes):
    out, i = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(theta[i:i + n].reshape(s))
        i += n
    return out


def flatten(arrs):
    return np.concatenate([np.asarray(a).ravel() for a in arrs])


def mlp_init(rng, shapes, gauss, last_scale=0.1):
    """glorot-uniform kernels, zero biases, last kernel x0.1, logstd 0 (`agentzoo.py:34-48`)."""
    arrs = []
    n_dense = (len(shapes) - (1 if gauss else 0)) // 2
    for i in range(n_dense):
        fi, fo = shapes[2 * i]
        lim = np.sqrt(6.0 / (fi + fo))
        W = rng.uniform(-lim, lim, size=(fi, fo))
        if i == n_dense - 1:
            W = W * last_scale
        arrs += [W, np.zeros(fo)]
    if gauss:
        arrs.append(np.zeros(shapes[-1]))
    return flatten(arrs)


class Spec:
    """Policy / value net shape.  head: 'softmax' (Categorical), 'gauss' (DiagGauss), 'linear' (VF)."""

    def __init__(self, n_in, hid, n_out, head):
        self.n_in, self.hid, self.n_out, self.head = n_in, list(hid), n_out, head
        self.shapes = mlp_shapes(n_in, self.hid, n_out, head == "gauss")
        self.P = n_params(self.shapes)

    def split(self, theta):
        arrs = unflatten(theta, self.shapes)
        logstd = arrs.pop() if self.head == "gauss" else None
        return arrs[0::2], arrs[1::2], logstd


def mlp_forward(spec, theta, x, dtype=np.float64):
    """Returns (z = pre-head output, acts=[x, h1, ..., hL])."""
    Ws, bs, _ = spec.split(theta.astype(dtype))
    h = np.asarray(x, dtype=dtype)
    acts = [h]
    for W, b in zip(Ws[:-1], bs[:-1]):
        h = np.tanh(h @ W + b)
        acts.append(h)
    z = h @ Ws[-1] + bs[-1]
    return z, acts


def softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def head_prob(spec, theta, z, dtype=np.float64):
    """prob rows: softmax(z) (`agentzoo.py:46`) or [mean, exp(logstd)] (`core.py:720-725`)."""
    if spec.head == "softmax":
        return softmax(z)
    if spec.head == "gauss":
        _, _, logstd = spec.split(theta.astype(dtype))
        std = np.repeat(np.exp(logstd)[None, :], z.shape[0], axis=0)
        return np.concatenate([z, std], axis=1)
    return z


def policy_prob(spec, theta, x, dtype=np.float64):
    z, _ = mlp_forward(spec, theta, x, dtype)
    return head_prob(spec, theta, z, dtype)


def mlp_vjp(spec, theta, acts, gz, dtype=np.float64):
    """Backprop gz = dL/dz through the tanh MLP; returns flat grads (no logstd slot)."""
    Ws, _, _ = spec.split(theta.astype(dtype))
    grads = []
    g = gz
    for l in reversed(range(len(Ws))):
        grads.append((acts[l].T @ g, g.sum(axis=0)))
        if l > 0:
            g = (g @ Ws[l].T) * (1 - acts[l] ** 2)
    out = []
    for gW, gb in reversed(grads):
        out += [gW, gb]
    return out


def mlp_jvp(spec, theta, dtheta, acts, dtype=np.float64):
    """Forward-mode derivative of z along dtheta (activations from the primal pass)."""
    Ws, _, _ = spec.split(theta.astype(dtype))
    dWs, dbs, _ = spec.split(dtheta.astype(dtype))
    dh = np.zeros_like(acts[0])
    for l in range(len(Ws)):
        da = dh @ Ws[l] + acts[l] @ dWs[l] + dbs[l]
        if l < len(Ws) - 1:
            dh = (1 - acts[l + 1] ** 2) * da
        else:
            return da


# ============================================================== probtypes
def loglik(spec, a, prob):
    """Categorical `core.py:349-353`; DiagGauss `core.py:412-416`."""
    if spec.head == "softmax":
        return np.log(prob[np.arange(prob.shape[0]), a.astype(np.int64)])
    d = spec.n_out
    m, s = prob[:, :d], prob[:, d:]
    return -0.5 * np.square((a - m) / s).sum(axis=1) - 0.5 * LOG2PI * d - np.log(s).sum(axis=1)


def kl(spec, p0, p1):
    """Categorical `core.py:355-356`; DiagGauss `core.py:421-426`."""
    if spec.head == "softmax":
        return (p0 * np.log(p0 / p1)).sum(axis=1)
    d = spec.n_out
    m0, s0, m1, s1 = p0[:, :d], p0[:, d:], p1[:, :d], p1[:, d:]
    return np.log(s1 / s0).sum(axis=1) + ((np.square(s0) + np.square(m0 - m1)) / (2.0 * np.square(s1))).sum(axis=1) - 0.5 * d


def entropy(spec, p):
    """Categorical `core.py:358-359`; DiagGauss `core.py:428-430`."""
    if spec.head == "softmax":
        return -(p * np.log(p)).sum(axis=1)
    d = spec.n_out
    return np.log(p[:, d:]).sum(axis=1) + 0.5 * np.log(2 * np.pi * np.e) * d


def sample(spec, prob, noise):
    """Categorical: argmax(cumsum(p) > u) (`distributions.py:3-13`);
    DiagGauss: z*std + mean, z cast to floatX (`core.py:432-435`).  noise = u[N] or z[N,d]."""
    if spec.head == "softmax":
        cs = np.cumsum(prob, axis=1)
        return np.argmax(cs > noise[:, None], axis=1)
    d = spec.n_out
    return noise.astype(prob.dtype) * prob[:, d:] + prob[:, :d]


# ============================================================== TRPO graph (trpo.py:29-70)
def surr_kl_ent(spec, theta, ob, act, adv, oldprob, dtype=np.float64):
    """losses [surr, kl, ent] (`trpo.py:42,60-64`)."""
    prob = policy_prob(spec, theta, ob, dtype)
    N = ob.shape[0]
    logp = loglik(spec, act, prob)
    oldlogp = loglik(spec, act, oldprob.astype(dtype))
    surr = (-1.0 / N) * np.exp(logp - oldlogp).dot(adv.astype(dtype))
    return np.array([surr, kl(spec, oldprob.astype(dtype), prob).mean(), entropy(spec, prob).mean()])


def policy_gradient(spec, theta, ob, act, adv, oldprob, dtype=np.float64):
    """pg = d surr / d theta (`trpo.py:42-43`), analytic backprop."""
    z, acts = mlp_forward(spec, theta, ob, dtype)
    prob = head_prob(spec, theta, z, dtype)
    N = ob.shape[0]
    ratio = np.exp(loglik(spec, act, prob) - loglik(spec, act, oldprob.astype(dtype)))
    w = (-1.0 / N) * ratio * adv.astype(dtype)
    if spec.head == "softmax":
        onehot = np.zeros_like(prob)
        onehot[np.arange(N), act.astype(np.int64)] = 1
        gz = w[:, None] * (onehot - prob)
        return flatten(mlp_vjp(spec, theta, acts, gz, dtype))
    d = spec.n_out
    m, s = prob[:, :d], prob[:, d:]
    u = (act - m) / s
    gz = w[:, None] * u / s
    glogstd = (w[:, None] * (u * u - 1.0)).sum(axis=0)
    return flatten(mlp_vjp(spec, theta, acts, gz, dtype) + [glogstd])


def fisher_vector_product(spec, theta, v, ob, dtype=np.float64):
    """Hessian of kl_firstfixed = sum KL(stopgrad(p), p)/N times v (`trpo.py:45-58`),
    evaluated in its exact Gauss-Newton form J^T M J v / N."""
    z, acts = mlp_forward(spec, theta, ob, dtype)
    N = ob.shape[0]
    dz = mlp_jvp(spec, theta, np.asarray(v), acts, dtype)
    if spec.head == "softmax":
        p = softmax(z)
        gz = p * (dz - (p * dz).sum(axis=1, keepdims=True)) / N
        return flatten(mlp_vjp(spec, theta, acts, gz, dtype))
    d = spec.n_out
    _, _, logstd = spec.split(theta.astype(dtype))
    var = np.exp(2 * logstd)
    _, _, dlogstd = spec.split(np.asarray(v).astype(dtype))
    gz = dz / var[None, :] / N
    return flatten(mlp_vjp(spec, theta, acts, gz, dtype) + [2.0 * dlogstd])


def cg(f_Ax, b, cg_iters=10, residual_tol=1e-10):
    """Demmel CG (`trpo.py:165-200`). Returns (x, iterations run, final rdotr)."""
    p = b.copy()
    r = b.copy()
    x = np.zeros_like(b)
    rdotr = r.dot(r)
    its = 0
    for _ in range(cg_iters):
        z = f_Ax(p)
        v = rdotr / p.dot(z)
        x += v * p
        r -= v * z
        newrdotr = r.dot(r)
        mu = newrdotr / rdotr
        p = r + mu * p
        rdotr = newrdotr
        its += 1
        if rdotr < residual_tol:
            break
    return x, its, rdotr


def linesearch(f, x, fullstep, expected_improve_rate, max_backtracks=10, accept_ratio=.1):
    """Backtracking line search (`trpo.py:143-159`). Returns (success, x, k, ratios, fvals)."""
    fval = f(x)
    ratios, fvals = [], [fval]
    for k, stepfrac in enumerate(.5 ** np.arange(max_backtracks)):
        xnew = x + stepfrac * fullstep
        newfval = f(xnew)
        fvals.append(newfval)
        actual_improve = fval - newfval
        expected_improve = expected_improve_rate * stepfrac
        ratio = actual_improve / expected_improve
        ratios.append(ratio)
        if ratio > accept_ratio and actual_improve > 0:
            return True, xnew, k, ratios, fvals
    return False, x, -1, ratios, fvals


class RowChunks:
    """The batch means of the TRPO graph (pg, Fvp, [surr, kl, ent]) evaluated over row
    chunks on a thread pool (numpy's BLAS calls and large ufuncs release the GIL), so the
    float64 oracle finishes at the benchmark's 4.19 M rows in seconds.  Every quantity
    of `trpo.py:29-70` is a mean over rows plus a row-independent term (the DiagGauss
    logstd parts), so the full-batch value is the chunk values weighted by n_c / N; the
    float64 sums differ from the one-pass evaluation only in summation order."""

    def __init__(self, ob, act, adv, oldprob, workers=16, chunk=1 << 18):
        from concurrent.futures import ThreadPoolExecutor
        self.n = ob.shape[0]
        self.sl = [slice(lo, min(lo + chunk, self.n)) for lo in range(0, self.n, chunk)]
        self.ob, self.act, self.adv, self.oldprob = ob, act, adv, oldprob
        self.pool = ThreadPoolExecutor(max_workers=workers)

    def _mean(self, fn):
        parts = list(self.pool.map(lambda s: fn(s) * ((s.stop - s.start) / self.n), self.sl))
        out = parts[0].astype(np.float64)
        for p in parts[1:]:
            out = out + p
        return out

    def pg(self, spec, theta, dtype=np.float64):
        return self._mean(lambda s: policy_gradient(spec, theta, self.ob[s], self.act[s], self.adv[s], self.oldprob[s],
                                                    dtype))

    def fvp(self, spec, theta, v, dtype=np.float64):
        return self._mean(lambda s: fisher_vector_product(spec, theta, v, self.ob[s], dtype))

    def losses(self, spec, theta, dtype=np.float64):
        return self._mean(lambda s: surr_kl_ent(spec, theta, self.ob[s], self.act[s], self.adv[s], self.oldprob[s],
                                                dtype))


def trpo_update(spec, theta, ob, act, adv, oldprob, cg_damping=1e-3, max_kl=1e-2, dtype=np.float64, rows=None):
    """TrpoUpdater.__call__ (`trpo.py:72-140`, HEAD diagnostics 82-84/97-100/131-132
    and the duplicate beta Fvp at 111 dropped).  Returns (theta_new, stats, diag).
    rows: a RowChunks over the same batch evaluates the graph's means chunk-parallel."""
    cast = (lambda t: t.astype(dtype))
    thprev = cast(theta)
    if rows is not None:
        def policy_gradient_(sp, th, _ob, _act, _adv, _oldprob, dt):
            return rows.pg(sp, th, dt)

        def surr_kl_ent_(sp, th, _ob, _act, _adv, _oldprob, dt):
            return rows.losses(sp, th, dt)

        def fisher_vector_product_(sp, th, v, _ob, dt):
            return rows.fvp(sp, th, v, dt)
    else:
        policy_gradient_, surr_kl_ent_, fisher_vector_product_ = policy_gradient, surr_kl_ent, fisher_vector_product
    g = policy_gradient_(spec, thprev, ob, act, adv, oldprob, dtype)
    losses_before = surr_kl_ent_(spec, thprev, ob, act, adv, oldprob, dtype)
    diag = {"g": g}
    th = thprev
    if np.allclose(g, 0):
        diag["skipped"] = True
    else:
        def fvp(p):
            # flat_tangent is a T.fvector (trpo.py:48): the tangent is downcast to floatX
            return fisher_vector_product_(spec, thprev, p.astype(dtype), ob, dtype).astype(np.float64) + cg_damping * p

        stepdir, its, rdotr = cg(fvp, -g.astype(np.float64))
        shs = .5 * stepdir.dot(fvp(stepdir))
        lm = np.sqrt(shs / max_kl)
        fullstep = stepdir / lm
        neggdotstepdir = -g.astype(np.float64).dot(stepdir)

        def loss(t):
            return surr_kl_ent_(spec, cast(t), ob, act, adv, oldprob, dtype)[0]

        success, theta_new, k, ratios, fvals = linesearch(loss, thprev.astype(np.float64), fullstep, neggdotstepdir / lm)
        th = cast(theta_new)  # SetFromFlat casts to floatX (core.py:540)
        diag.update(stepdir=stepdir, cg_iters=its, rdotr=rdotr, shs=shs, lm=lm, fullstep=fullstep,
                    neggdotstepdir=neggdotstepdir, success=success, k=k, ratios=np.array(ratios),
                    fvals=np.array(fvals), skipped=False)
    losses_after = surr_kl_ent_(spec, th, ob, act, adv, oldprob, dtype)
    stats = OrderedDict()
    for name, lb, la in zip(["surr", "kl", "ent"], losses_before, losses_after):
        stats[name + "_before"] = lb
        stats[name + "_after"] = la
    return th, stats, diag


# ============================================================== advantage (core.py:63-105)
def compute_advantage(vf_predict, paths, gamma, lam):
    """Per-path GAE + return + batch standardisation (`core.py:63-105`, TF check 79-96 dropped)."""
    for path in paths:
        path["return"] = discount(path["reward"], gamma)
        b = path["baseline"] = vf_predict(path)
        b1 = np.append(b, 0 if path["terminated"] else b[-1])
        deltas = path["reward"] + gamma * b1[1:] - b1[:-1]
        path["advantage"] = discount(deltas, gamma * lam)
    alladv = np.concatenate([path["advantage"] for path in paths])
    std = alladv.std()
    mean = alladv.mean()
    for path in paths:
        path["advantage"] = (path["advantage"] - mean) / std


def gae_batched(rew, v, last, term, gamma, lam):
    """Time-major [T,E] form of the per-path recursion above (row flags: last = episode
    ends at this row (done or horizon/timestep-limit cut), term = ended by env done).
    Returns (adv_unstandardised, ret)."""
    T, E = rew.shape
    adv = np.zeros((T, E))
    ret = np.zeros((T, E))
    a_next = np.zeros(E)
    r_next = np.zeros(E)
    v_next = np.zeros(E)
    for t in reversed(range(T)):
        cont = ~last[t]
        boot = np.where(cont, v_next, np.where(term[t], 0.0, v[t]))
        delta = rew[t] + gamma * boot - v[t]
        a_next = delta + gamma * lam * np.where(cont, a_next, 0.0)
        r_next = rew[t] + gamma * np.where(cont, r_next, 0.0)
        adv[t] = a_next
        ret[t] = r_next
        v_next = v[t]
    return adv, ret


def standardize(x):
    """(x - mean) / std with numpy std, ddof=0, no epsilon (`core.py:100-105`)."""
    return (x - x.mean()) / x.std()


# ============================================================== value function (core.py:595-697)
VF_L2 = 1e-3


def vf_loss_grad(spec, theta, X, y, dtype=np.float64):
    """loss = sum((y - yhat)^2)/N + 1e-3 * sum(theta^2) (`core.py:611-617`) and its flat grad."""
    th = theta.astype(dtype)
    z, acts = mlp_forward(spec, th, X, dtype)
    N = X.shape[0]
    err = z - y.reshape(-1, 1).astype(dtype)
    mse = np.sum(np.square(err)) / N
    l2 = VF_L2 * np.sum(np.square(th))
    g = flatten(mlp_vjp(spec, th, acts, 2.0 * err / N, dtype)) + 2.0 * VF_L2 * th
    return mse + l2, g, mse, l2


def vf_fit(spec, theta, X, ytarg, mixfrac=0.1, maxiter=2, dtype=np.float64):
    """NnRegression.fit + LbfgsOptimizer.update (`core.py:620-637, 674-697`)."""
    predict = (lambda t: mlp_forward(spec, t, X, dtype)[0])
    th0 = theta.astype(dtype)
    ypredold = predict(th0)
    target = ytarg.reshape(-1, 1) * mixfrac + ypredold * (1 - mixfrac)

    def lossandgrad(t):
        l, g, _, _ = vf_loss_grad(spec, t.astype(dtype), X, target, dtype)
        return float(l), g.astype(np.float64)

    lb, _, mb, l2b = vf_loss_grad(spec, th0, X, target, dtype)
    th, _, info = scipy.optimize.fmin_l_bfgs_b(lossandgrad, th0.astype(np.float64), maxiter=maxiter)
    th = th.astype(dtype)
    la, _, ma, l2a = vf_loss_grad(spec, th, X, target, dtype)
    yprednew = predict(th)
    out = OrderedDict()
    out["loss_before"], out["loss_after"] = lb, la
    out["mse_before"], out["mse_after"] = mb, ma
    out["l2_before"], out["l2_after"] = l2b, l2a
    out["PredStdevBefore"] = ypredold.std()
    out["PredStdevAfter"] = yprednew.std()
    out["TargStdev"] = ytarg.std()
    out["EV_before"] = explained_variance_2d(ypredold, ytarg.reshape(-1, 1))[0]
    out["EV_after"] = explained_variance_2d(yprednew, ytarg.reshape(-1, 1))[0]
    return th, out, info, target


# ============================================================== stats (core.py:31-44)
def add_episode_stats(stats, paths):
    episoderewards = np.array([path["reward"].sum() for path in paths])
    pathlengths = np.array([len(path["reward"]) for path in paths])
    stats["EpisodeRewards"] = episoderewards
    stats["EpisodeLengths"] = pathlengths
    stats["NumEpBatch"] = len(episoderewards)
    stats["EpRewMean"] = episoderewards.mean()
    stats["EpRewSEM"] = episoderewards.std() / np.sqrt(len(paths))
    stats["EpRewMax"] = episoderewards.max()
    stats["EpLenMean"] = pathlengths.mean()
    stats["EpLenMax"] = pathlengths.max()
    stats["RewPerStep"] = episoderewards.sum() / pathlengths.sum()
