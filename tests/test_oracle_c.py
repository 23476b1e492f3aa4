"""oracle/mlp_c.c (the C restatement of the TRPO graph's batch means that the full-size
GPU tests use as their float64 truth) against the numpy oracle it restates: pg, the
Fisher product and the loss means to 1e-12, across heads, widths, depths, thread
counts and the activation cache; and the C-backed trpo_update against the numpy one."""
import numpy as np
import pytest

from oracle import trpo_c as C
from oracle import trpo_np as T


def _case(rng, head, nin, nout, hid, N):
    spec = T.Spec(nin, hid, nout, head)
    th = T.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
    if head == "gauss":
        th[-nout:] = 0.3 * rng.standard_normal(nout)
    ob = rng.standard_normal((N, nin))
    oldprob = T.policy_prob(spec, th + 0.01 * rng.standard_normal(spec.P), ob)
    act = T.sample(spec, oldprob, rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N))
    adv = rng.standard_normal(N)
    return spec, th, ob, act, adv, oldprob


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.mark.parametrize("head,nin,nout,hid", [("gauss", 11, 3, [64, 64]), ("softmax", 4, 2, [64, 64]),
                                               ("gauss", 17, 5, [32, 48, 40]), ("softmax", 6, 7, [20]),
                                               ("gauss", 376, 17, [512, 512, 512])])
@pytest.mark.parametrize("threads", [1, 5])
def test_c_oracle_matches_numpy(head, nin, nout, hid, threads):
    rng = np.random.default_rng(nin * 31 + nout)
    N = 300 if hid[0] == 512 else 2003
    spec, th, ob, act, adv, oldprob = _case(rng, head, nin, nout, hid, N)
    v = rng.standard_normal(spec.P)
    cr = C.CRows(spec, ob, act, adv, oldprob, threads=threads)
    assert _rel(cr.pg(spec, th), T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 1e-12
    want = T.fisher_vector_product(spec, th, v, ob)
    assert _rel(cr.fvp(spec, th, v), want) < 1e-12
    assert _rel(cr.fvp(spec, th, v), want) < 1e-12  # from the activation cache
    assert _rel(cr.losses(spec, th), T.surr_kl_ent(spec, th, ob, act, adv, oldprob)) < 1e-12
    th2 = th + 0.01 * rng.standard_normal(spec.P)  # a new theta refills the cache
    assert _rel(cr.fvp(spec, th2, v), T.fisher_vector_product(spec, th2, v, ob)) < 1e-12


@pytest.mark.parametrize("head,nin,nout", [("gauss", 11, 3), ("softmax", 4, 2)])
def test_c_backed_trpo_update_matches_numpy(head, nin, nout):
    rng = np.random.default_rng(5)
    spec, th, ob, act, adv, oldprob = _case(rng, head, nin, nout, [64, 64], 20000)
    a = T.trpo_update(spec, th, ob, act, adv, oldprob, cg_damping=0.1, max_kl=0.01)
    b = T.trpo_update(spec, th, ob, act, adv, oldprob, cg_damping=0.1, max_kl=0.01,
                      rows=C.CRows(spec, ob, act, adv, oldprob, threads=4))
    assert a[2]["k"] == b[2]["k"]
    assert np.abs(a[0] - b[0]).max() <= 1e-9 * np.abs(a[0] - th).max()
    np.testing.assert_allclose([b[2]["lm"], b[2]["shs"]], [a[2]["lm"], a[2]["shs"]], rtol=1e-10)
    for k in a[1]:
        np.testing.assert_allclose(b[1][k], a[1][k], rtol=1e-9, atol=1e-12)


def test_chunked_numpy_rows_match_one_pass():
    rng = np.random.default_rng(9)
    spec, th, ob, act, adv, oldprob = _case(rng, "gauss", 11, 3, [64, 64], 5000)
    rows = T.RowChunks(ob, act, adv, oldprob, workers=3, chunk=777)
    v = rng.standard_normal(spec.P)
    assert _rel(rows.pg(spec, th), T.policy_gradient(spec, th, ob, act, adv, oldprob)) < 1e-12
    assert _rel(rows.fvp(spec, th, v), T.fisher_vector_product(spec, th, v, ob)) < 1e-12
    assert _rel(rows.losses(spec, th), T.surr_kl_ent(spec, th, ob, act, adv, oldprob)) < 1e-12
