"""CPU checks of the Hopper-v2 articulated-body restatement (oracle/envs.py).

MuJoCo is absent, so the model is checked against physics instead of MuJoCo
output (parity with MuJoCo is unpinned): the mass matrix and bias terms conserve
energy in contact-free flight with the integrator's first-order error (halving dt
halves the drift), M is symmetric positive definite, and a standing hopper under
zero torque rests on its foot at the expected height.
"""
import numpy as np
import pytest

from oracle import envs as EV


def _mass_matrix_and_energy(q, v):
    qs = [q[:, i] for i in range(6)]
    qd = [v[:, i] for i in range(6)]
    phi = [qs[2]]
    for j in range(1, 4):
        phi.append(phi[j - 1] - qs[2 + j])
    sg = [np.sin(p) for p in phi]
    cg = [np.cos(p) for p in phi]
    B = [EV.hopper_body_terms(k, qs, qd, sg, cg) for k in range(4)]
    tot = [(B[0][t] + B[1][t]) + (B[2][t] + B[3][t]) for t in range(21)]
    E = q.shape[0]
    M = np.zeros((E, 6, 6))
    for n, (a, b) in enumerate(EV.HP_TRI):
        M[:, a, b] = tot[n]
        M[:, b, a] = tot[n]
    for j in (3, 4, 5):
        M[:, j, j] += EV.HP_ARM
    ke = 0.5 * np.einsum("ei,eij,ej->e", v, M, v)
    pe = np.zeros(E)
    pz = qs[1]
    for k in range(4):
        _, ez = EV._rot(sg[k], cg[k], *EV.HP_COM[k])
        pe = pe + EV.HP_MASS[k] * EV.HP_GRAV * (pz + ez)
        if k < 3:
            pz = pz - EV.HP_SEG[k] * cg[k]
    return M, ke + pe


@pytest.fixture
def free_flight(monkeypatch):
    monkeypatch.setattr(EV, "HP_DAMP", 0.0)
    monkeypatch.setattr(EV, "HP_LO", (-9.0, -9.0, -9.0))
    monkeypatch.setattr(EV, "HP_HI", (9.0, 9.0, 9.0))
    monkeypatch.setattr(EV, "HP_GRAV", 0.0)
    rng = np.random.default_rng(1)
    q = np.zeros((8, 6))
    q[:, 1] = 50.0  # far above the floor: no contact
    q[:, 2:] = rng.uniform(-0.5, 0.5, (8, 4))
    v = rng.uniform(-2, 2, (8, 6))
    return q, v


def test_energy_drift_is_first_order_in_dt(free_flight, monkeypatch):
    q0, v0 = free_flight
    M, e0 = _mass_matrix_and_energy(q0, v0)
    assert np.allclose(M, np.swapaxes(M, 1, 2))
    assert (np.linalg.eigvalsh(M) > 0).all()
    drift = []
    for dt, n in ((0.002, 250), (0.001, 500)):
        monkeypatch.setattr(EV, "HP_DT", dt)
        q, v = q0.copy(), v0.copy()
        for _ in range(n):
            q, v = EV._hopper_substep(q, v, np.zeros((8, 3)))
        drift.append(np.abs(_mass_matrix_and_energy(q, v)[1] - e0) / e0)
    assert drift[0].max() < 5e-3
    ratio = drift[0] / np.maximum(drift[1], 1e-15)
    assert np.all((ratio > 1.6) & (ratio < 2.5)), ratio


def test_hopper_rests_on_foot_and_random_policy_falls():
    rng = np.random.default_rng(0)
    E = 16
    q, v = EV.hopper_reset(rng.random((E, 12)))
    for _ in range(40):
        q, v, rew, done = EV.hopper_step(q, v, np.zeros((E, 3)))
    assert not done.any()
    # the foot capsule (radius .06) rests on the floor: torso centre 1.25 - 0.04 drop
    assert np.all(np.abs(q[:, 1] - 1.206) < 0.01), q[:, 1]
    assert np.all(np.abs(rew - 1.0) < 0.2)
    # a random policy topples within a few dozen steps (health test z > .7, |ang| < .2)
    q, v = EV.hopper_reset(rng.random((E, 12)))
    alive = np.ones(E, bool)
    for _ in range(200):
        q, v, rew, done = EV.hopper_step(q, v, rng.standard_normal((E, 3)))
        alive &= ~done
    assert not alive.any()


def test_recursive_form_matches_per_body_form():
    """The recursive CRBA/RNEA substep the device kernel mirrors equals the
    body-by-body assembly of M and tau_c - h (an independent formulation)."""
    rng = np.random.default_rng(3)
    E = 256
    q = np.zeros((E, 6))
    q[:, 0] = rng.normal(size=E)
    q[:, 1] = rng.uniform(0.9, 1.3, E)  # some states in ground contact
    q[:, 2:] = rng.uniform(-1, 1, (E, 4))
    v = rng.normal(size=(E, 6)) * 2
    tau = rng.normal(size=(E, 3)) * 100
    _, v1 = EV._hopper_substep_per_body(q, v, tau)
    _, v2 = EV._hopper_substep(q, v, tau)
    acc1, acc2 = (v1 - v) / EV.HP_DT, (v2 - v) / EV.HP_DT
    rel = np.abs(acc1 - acc2).max(axis=1) / np.abs(acc1).max(axis=1)
    assert rel.max() < 1e-11, rel.max()
