"""numpy restatement of the lock-step batched collector -- TEST INFRASTRUCTURE (oracle).

Follows the reference's per-step loop (`core.py:182-207`: obfilt -> act -> step ->
rewfilt) for E envs in lock-step, with the batched-filter rule of SURVEY Appendix
A.1 (all E observations of a step merged into the running stat -- as per-block
Welford partials in block order -- then normalised).  For E = 1 this is exactly
the reference's sequence of RunningStat.push calls.  Mirrors
``modular_rl_amd/csrc/rollout.hip`` step for step so the GPU collector can be
checked row by row; the policy forward here is float64 on the stored float32
observations.
"""
import numpy as np

from . import envs as EV
from . import philox
from . import trpo_np as T

BLOCK = 128
CARTPOLE, HOPPER, HUMANOID = 0, 1, 2


class FilterState:
    """(n, M, S) for the obs dims and the reward (the last column)."""

    def __init__(self, D):
        self.n = 0.0
        self.nr = 0.0
        self.M = np.zeros(D)
        self.S = np.zeros(D)

    def copy(self):
        f = FilterState(len(self.M))
        f.n, f.nr, f.M, f.S = self.n, self.nr, self.M.copy(), self.S.copy()
        return f


def _merge(n, M, S, nb, mb, m2b):
    if nb <= 0:
        return n, M, S
    nn = n + nb
    delta = mb - M
    newM = M + (delta * nb) / nn
    S = S + m2b + delta * (mb - newM) * nb
    return nn, newM, S


def _block_partials(vals):
    """vals [E, D] -> list of (n, mean[D], M2[D]) per block of BLOCK envs (sequential sums)."""
    out = []
    for b0 in range(0, vals.shape[0], BLOCK):
        v = vals[b0:b0 + BLOCK]
        n = v.shape[0]
        s = np.zeros(v.shape[1])
        for i in range(n):
            s = s + v[i]
        mean = s / n
        m2 = np.zeros(v.shape[1])
        for i in range(n):
            d = v[i] - mean
            m2 = m2 + d * d
        out.append((float(n), mean, m2))
    return out


def _batch(recs, col_sel, count_of):
    """Combine block records into one batch: n = sum n_b, mean = sum n_b mean_b / n,
    M2 = sum (M2_b + n_b (mean_b - mean)^2) -- the parallel form of Chan's merge."""
    n = sum(count_of(r) for r in recs)
    if n <= 0:
        return 0.0, 0.0, 0.0
    mean = sum(count_of(r) * col_sel(r[1]) for r in recs) / n
    m2 = sum(col_sel(r[2]) + count_of(r) * (col_sel(r[1]) - mean) ** 2 for r in recs if count_of(r) > 0)
    return n, mean, m2


def _merge_records(fs, recs, with_obs=True, with_rew=True):
    D = len(fs.M)
    O = D - 1
    bn, bm, bs = _batch(recs, lambda v: v, lambda r: r[0])
    bnr, bmr, bsr = _batch(recs, lambda v: v[O], lambda r: r[0] if r[3] else 0.0)
    if with_obs:
        n, M, S = _merge(fs.n, fs.M[:O], fs.S[:O], bn, bm[:O], bs[:O])
        fs.n, fs.M[:O], fs.S[:O] = n, M, S
    if with_rew:
        nr, Mr, Sr = _merge(fs.nr, fs.M[O], fs.S[O], bnr, bmr, bsr)
        fs.nr, fs.M[O], fs.S[O] = nr, Mr, Sr
    return fs


class Envs:
    def __init__(self, kind, E, seed, env_offset=0):
        self.kind, self.E, self.seed = kind, E, seed
        self.gid = np.arange(E, dtype=np.uint64) + np.uint64(env_offset)
        self.ns, self.O, self.A, self.max_steps, self.nu = {
            CARTPOLE: (4, 4, 2, 200, 4), HOPPER: (12, 11, 3, 1000, 12),
            HUMANOID: (EV.HM_NS, EV.HM_OBS, EV.HM_ACT, 1000, EV.HM_NU)}[kind]
        self.state = np.zeros((E, self.ns))
        self.ep_t = np.zeros(E, dtype=np.int64)
        self.ep_count = np.zeros(E, dtype=np.int64)

    def reset(self, idx):
        u = philox.uniforms(self.seed, 1, self.gid[idx], self.ep_count[idx].astype(np.uint64), self.nu)
        if self.kind == CARTPOLE:
            self.state[idx] = EV.cartpole_reset(u)
        elif self.kind == HUMANOID:
            self.state[idx] = EV.humanoid_reset(u)
        else:
            q, v = EV.hopper_reset(u)
            self.state[idx] = np.concatenate([q, v], axis=1)
        self.ep_count[idx] += 1
        self.ep_t[idx] = 0

    def obs(self):
        if self.kind == CARTPOLE:
            return self.state.copy()
        if self.kind == HUMANOID:
            return EV.humanoid_obs(self.state)
        return EV.hopper_obs(self.state[:, :6], self.state[:, 6:])

    def step(self, act):
        if self.kind == CARTPOLE:
            s2, rew, done = EV.cartpole_step(self.state, act)
            self.state = s2
        elif self.kind == HUMANOID:
            self.state, rew, done = EV.humanoid_step(self.state, act)
        else:
            q, v, rew, done = EV.hopper_step(self.state[:, :6], self.state[:, 6:], act)
            self.state = np.concatenate([q, v], axis=1)
        return rew, done


def collect(envs, fs, spec, theta, Tn, timestep_limit, iteration, filt=True, noise=None):
    """One iteration: reset all envs, Tn lock-step steps.  Returns trajectory dict
    (time-major [Tn, E, ...]) and updates envs / fs in place."""
    E, O, A = envs.E, envs.O, envs.A
    envs.reset(np.arange(E))
    o = envs.obs()
    recs = [(n, m, m2, False) for (n, m, m2) in _block_partials(np.concatenate([o, np.zeros((E, 1))], axis=1))]
    out = dict(obs=np.zeros((Tn, E, O), np.float32), rew=np.zeros((Tn, E), np.float32),
               flags=np.zeros((Tn, E), np.uint8), ep_t=np.zeros((Tn, E), np.int32),
               act=np.zeros((Tn, E), np.int32) if spec.head == "softmax" else np.zeros((Tn, E, A), np.float32),
               prob=np.zeros((Tn, E, A if spec.head == "softmax" else 2 * A), np.float32))
    for t in range(Tn):
        fs = _merge_records(fs, recs)
        o = envs.obs()
        if filt:
            var = fs.S[:O] / (fs.n - 1) if fs.n > 1 else fs.M[:O] ** 2
            x = np.clip((o - fs.M[:O]) / (np.sqrt(var) + 1e-8), -5.0, 5.0)
        else:
            x = o
        x32 = x.astype(np.float32)
        out["obs"][t] = x32
        z, _ = T.mlp_forward(spec, theta, x32.astype(np.float64))
        w = np.uint64(iteration * Tn + t)
        if spec.head == "softmax":
            p = T.softmax(z).astype(np.float32)
            u = noise[t] if noise is not None else philox.uniform2(envs.seed, 0, envs.gid, w, 0)[0]
            cs = np.cumsum(p, axis=1, dtype=np.float32)
            act = np.argmax(cs.astype(np.float64) > u[:, None], axis=1)
            out["prob"][t] = p
        else:
            _, _, logstd = spec.split(theta)
            sd = np.exp(logstd.astype(np.float32))
            zn = noise[t] if noise is not None else philox.normals(envs.seed, 0, envs.gid, w, A)
            act = zn.astype(np.float32) * sd[None, :] + z.astype(np.float32)
            out["prob"][t] = np.concatenate([z.astype(np.float32), np.repeat(sd[None, :], E, axis=0)], axis=1)
        out["act"][t] = act
        rew, done = envs.step(act)
        ept = envs.ep_t.copy()
        out["ep_t"][t] = ept
        term = done | (ept + 1 >= envs.max_steps)
        last = term | (ept + 1 >= timestep_limit) | (t == Tn - 1)
        out["rew"][t] = rew.astype(np.float32)
        out["flags"][t] = last.astype(np.uint8) | (term.astype(np.uint8) << 1)
        envs.ep_t = ept + 1
        if t < Tn - 1 and last.any():
            envs.reset(np.nonzero(last)[0])
        o2 = envs.obs()
        recs = [(n, m, m2, True) for (n, m, m2) in
                _block_partials(np.concatenate([o2, rew[:, None]], axis=1))]
    fs = _merge_records(fs, recs, with_obs=False, with_rew=True)
    return out, fs
