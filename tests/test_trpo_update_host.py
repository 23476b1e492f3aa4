"""TrpoUpdater.update host logic on the float64 oracle ops (CPU, one rank).

* a zero policy gradient (all advantages 0) skips the update (`trpo.py:115-117`):
  theta untouched, losses_after == losses_before, although the first line-search
  batch was already issued (on a NaN full step) ahead of the readback;
* the batched line search with its first batch fused into the post-CG readback takes
  the same step as the serial one-candidate loop.
"""
import types

import numpy as np

from oracle import trpo_np as T
from tests.test_dist_gloo import _data


def _updater(th, spec, batches):
    from modular_rl_amd.dist import Comm
    from modular_rl_amd.trpo import TrpoUpdater
    from tests.oracle_ops import OracleOps, fake_policy
    pol = fake_policy(spec, th)
    up = TrpoUpdater(pol, dict(cg_damping=0.1, max_kl=0.01), comm=Comm(), ops=OracleOps(spec, pol.net))
    up.LS_BATCHES = batches
    return pol, up


def test_zero_gradient_skips_update():
    spec, th, ob, act, adv, oldprob = _data(N=200)
    pol, up = _updater(th, spec, (1, 3, 6))
    th0 = pol.net.theta.numpy().copy()
    b = types.SimpleNamespace(n=len(ob), obs=ob, act=act, adv=np.zeros_like(adv), prob=oldprob)
    with np.errstate(all="ignore"):
        stats = up.update(b)
    assert up.last_diag["skipped"] is True
    np.testing.assert_array_equal(pol.net.theta.numpy(), th0)
    for name in ("surr", "kl", "ent"):
        assert stats[name + "_after"] == stats[name + "_before"]


def test_fused_first_batch_equals_serial_linesearch():
    spec, th, ob, act, adv, oldprob = _data(N=300)
    b = types.SimpleNamespace(n=len(ob), obs=ob, act=act, adv=adv, prob=oldprob)
    out = []
    for batches in ((1, 3, 6), None):
        pol, up = _updater(th, spec, batches)
        stats = up.update(b)
        out.append((pol.net.theta.numpy().copy(), dict(stats), up.last_diag["k"], up.last_diag["ls"]))
    (th_b, st_b, k_b, ls_b), (th_s, st_s, k_s, ls_s) = out
    assert k_b == k_s
    np.testing.assert_array_equal(th_b, th_s)
    np.testing.assert_array_equal(ls_b, ls_s)
    for k in st_s:
        assert st_b[k] == st_s[k]
