"""The reference's own known-answer checks, run against the HIP kernels.

* ``validate_probtype`` (core.py:440-483): for the reference's DiagGauss and
  Categorical test distributions, Monte-Carlo over N = 100,000 samples, the mean
  negative log-likelihood equals the entropy and ``-ent[p] - E_p[log q]`` equals
  ``kl[p, q]``, each within 3 standard errors.  loglik / kl / entropy come from
  mrl_probtype_rows, i.e. the fp32 device helpers the MLP row epilogues (surrogate,
  KL and entropy of the TRPO losses) are built from; the samples are drawn on the
  host exactly as the reference draws them (np.random.seed(0), then
  ``probtype.sample``).
* A CartPole-v0 step against gym's classic-control equations written out here
  (independent of oracle/envs.py), pinned first to a hand-computed transition.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def _probtype_rows(head, k, prob, prob2=None, x=None):
    from modular_rl_amd import _lib
    from modular_rl_amd._lib import call, ptr, stream
    n = prob.shape[0]
    pd = _dev(prob)
    p2 = _dev(prob2) if prob2 is not None else None
    xd = None
    if x is not None:
        xd = _dev(x, torch.int32) if head == _lib.HEAD_SOFTMAX else _dev(x)
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)]
    ll, kl, ent = (outs[0] if x is not None else None), (outs[1] if prob2 is not None else None), outs[2]
    call("mrl_probtype_rows", int(head), int(k), int(n), ptr(pd), ptr(p2), ptr(xd), ptr(ll), ptr(kl), ptr(ent),
         stream())
    torch.cuda.synchronize()
    return [None if o is None else o.cpu().numpy().astype(np.float64) for o in (ll, kl, ent)]


def _validate_probtype(head, k, prob, sample):
    """core.py:457-483 with the Theano functions replaced by mrl_probtype_rows."""
    N = 100000
    Mval = np.repeat(prob[None, :], N, axis=0)
    Xval = sample(Mval)
    logliks, _, ents = _probtype_rows(head, k, Mval, x=Xval)
    entval_ll = -logliks.mean()
    entval_ll_stderr = logliks.std() / np.sqrt(N)
    entval = ents.mean()
    assert np.abs(entval - entval_ll) < 3 * entval_ll_stderr, (entval, entval_ll, entval_ll_stderr)
    q = prob + np.random.randn(prob.size) * 0.1
    Mval2 = np.repeat(q[None, :], N, axis=0)
    _, kls, _ = _probtype_rows(head, k, Mval, prob2=Mval2)
    klval = kls.mean()
    logliks2, _, _ = _probtype_rows(head, k, Mval2, x=Xval)
    klval_ll = -entval - logliks2.mean()
    klval_ll_stderr = logliks2.std() / np.sqrt(N)
    assert np.abs(klval - klval_ll) < 3 * klval_ll_stderr, (klval, klval_ll, klval_ll_stderr)
    return entval, klval


def test_validate_probtype_diag_gauss_and_categorical():
    """test_probtypes (core.py:440-455): one seed, DiagGauss first, then Categorical."""
    from modular_rl_amd import _lib
    np.random.seed(0)
    prob_diag_gauss = np.array([-.2, .3, .4, -.5, 1.1, 1.5, .1, 1.9])
    d = prob_diag_gauss.size // 2

    def gauss_sample(M):  # DiagGauss.sample (core.py:432-435)
        return np.random.randn(M.shape[0], d) * M[:, d:] + M[:, :d]

    ent_g, kl_g = _validate_probtype(_lib.HEAD_GAUSS, d, prob_diag_gauss, gauss_sample)
    # closed forms of the same quantities (core.py:421-430), float64
    s = prob_diag_gauss[d:]
    assert abs(ent_g - (np.log(s).sum() + 0.5 * d * np.log(2 * np.pi * np.e))) < 1e-5 * abs(ent_g) + 1e-6

    prob_categorical = np.array([.2, .3, .5])

    def cat_sample(M):  # categorical_sample (distributions.py:3-13)
        cs = np.cumsum(M, axis=1)
        return np.argmax(cs > np.random.rand(M.shape[0], 1), axis=1)

    ent_c, _ = _validate_probtype(_lib.HEAD_SOFTMAX, 3, prob_categorical, cat_sample)
    assert abs(ent_c + (prob_categorical * np.log(prob_categorical)).sum()) < 1e-6


# ----------------------------------------------------------------- CartPole-v0
GRAVITY, MASSCART, MASSPOLE, LENGTH, FORCE_MAG, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
TOTAL_MASS = MASSPOLE + MASSCART
POLEMASS_LENGTH = MASSPOLE * LENGTH
THETA_LIMIT = 12 * 2 * math.pi / 360


def gym_cartpole_step(state, action):
    """gym/envs/classic_control/cartpole.py (the version CartPole-v0 registers): Euler."""
    x, x_dot, theta, theta_dot = state
    force = FORCE_MAG if action == 1 else -FORCE_MAG
    costheta, sintheta = math.cos(theta), math.sin(theta)
    temp = (force + POLEMASS_LENGTH * theta_dot * theta_dot * sintheta) / TOTAL_MASS
    thetaacc = (GRAVITY * sintheta - costheta * temp) / (LENGTH * (4.0 / 3.0 - MASSPOLE * costheta ** 2 / TOTAL_MASS))
    xacc = temp - POLEMASS_LENGTH * thetaacc * costheta / TOTAL_MASS
    nxt = (x + TAU * x_dot, x_dot + TAU * xacc, theta + TAU * theta_dot, theta_dot + TAU * thetaacc)
    done = nxt[0] < -2.4 or nxt[0] > 2.4 or nxt[2] < -THETA_LIMIT or nxt[2] > THETA_LIMIT
    return nxt, 1.0, done


def test_cartpole_equations_hand_computed():
    """From rest with action 1: temp = 10 / 1.1, thetaacc = -temp / (0.5 (4/3 - 0.1/1.1)),
    xacc = temp - 0.05 thetaacc / 1.1, worked by hand."""
    nxt, r, done = gym_cartpole_step((0.0, 0.0, 0.0, 0.0), 1)
    temp = 10.0 / 1.1
    thetaacc = -temp / (0.5 * (4.0 / 3.0 - 0.1 / 1.1))   # -14.634146...
    xacc = temp - 0.05 * thetaacc / 1.1                  # 9.756097...
    assert abs(thetaacc + 14.634146341463415) < 1e-12 and abs(xacc - 9.75609756097561) < 1e-12
    np.testing.assert_allclose(nxt, (0.0, 0.02 * xacc, 0.0, 0.02 * thetaacc), rtol=0, atol=1e-15)
    assert r == 1.0 and not done


def test_cartpole_device_steps_follow_gym_equations():
    """Unfiltered CartPole rollout on the device: every stored transition (obs_t,
    act_t) -> obs_{t+1} of an unfinished episode equals gym's equations applied to
    obs_t (fp32 rows), reward 1 every step, and the terminated flag set exactly when
    the next state leaves the 2.4 / 12-degree box or the 200-step TimeLimit ends it."""
    from modular_rl_amd.collector import Collector
    from modular_rl_amd.envs import make
    from tests.test_gpu_pipeline import _policy
    env = make("CartPole-v0")
    _, _, pol = _policy("softmax", 4, 2, seed=21)
    E, Tn = 64, 300
    col = Collector(env, pol, E, Tn, 200, filter=0, seed=5, use_graph=False)
    b = col.collect()
    obs = b.obs.cpu().numpy().reshape(Tn, E, 4).astype(np.float64)
    act = b.act.cpu().numpy().reshape(Tn, E)
    rew = b.rew.cpu().numpy().reshape(Tn, E)
    flags = b.flags.cpu().numpy().reshape(Tn, E)
    ep_t = b.ep_t.cpu().numpy().reshape(Tn, E)
    assert np.all(rew == 1.0)
    checked = terminations = 0
    for e in range(E):
        for t in range(Tn):
            nxt, _, done = gym_cartpole_step(obs[t, e], int(act[t, e]))
            timelimit = ep_t[t, e] + 1 >= 200
            if t + 1 < Tn:
                term = bool(flags[t, e] & 2)
                # a transition within 1e-6 of the box edge could round either way from fp32 rows
                near = min(abs(abs(nxt[0]) - 2.4), abs(abs(nxt[2]) - THETA_LIMIT)) < 1e-5
                if not near:
                    assert term == (done or timelimit), (e, t, nxt, flags[t, e])
                terminations += int(done)
            if not flags[t, e] & 1:
                np.testing.assert_allclose(obs[t + 1, e], nxt, rtol=2e-6, atol=2e-6, err_msg=f"env {e} step {t}")
                checked += 1
    assert checked > E * Tn // 2 and terminations > 0
