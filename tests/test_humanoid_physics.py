"""Physics checks of the Humanoid-v2 restatement (oracle/humanoid.py; the HIP step is
its twin, tests/test_gpu_humanoid.py).  MuJoCo is absent, so the dynamics are pinned
by invariants rather than by MuJoCo output:

* the CRBA mass matrix equals an independent assembly from finite-difference body
  Jacobians (sum_b m J_v^T J_v + J_w^T I_w J_w + armature) and is positive definite;
* in free fall, whatever the internal forces (motors, springs, damping, limits), the
  accelerations the solver returns make the linear momentum change at -M g and the
  angular momentum about the COM stay constant (central differences along the
  trajectory);
* with damping off and no contact, energy drift is first order in dt;
* a random policy (U(-0.4, 0.4) controls) ends its episodes after ~22 steps as
  Humanoid-v2 under MuJoCo does, and a fallen humanoid comes to rest on the floor.
"""
import numpy as np
import pytest

from oracle import humanoid as H
from modular_rl_amd.humanoid_model import MODEL, NB, NV


def _states(E, seed, z=None, spread=0.3):
    rng = np.random.default_rng(seed)
    s = H.humanoid_reset(rng.random((E, H.NU)))
    q, qd = s[:, :H.NQ].copy(), s[:, H.NQ:H.NQ + NV].copy()
    quat = rng.standard_normal((E, 4))
    q[:, 3:7] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
    lo, hi = MODEL["hinge_lo"], MODEL["hinge_hi"]
    q[:, 7:] = lo + (hi - lo) * rng.uniform(0.2, 0.8, (E, 17))
    qd = rng.standard_normal((E, NV)) * spread
    if z is not None:
        q[:, 2] = z
    return q, qd, rng


def test_model_mass_properties():
    m = MODEL["body_mass"]
    assert 38.0 < m.sum() < 45.0  # gym's Humanoid-v2 weighs about 40 kg
    assert np.all(m > 1.0)
    for b in range(NB):
        I6 = MODEL["body_inertia"][b]
        I = np.array([[I6[0], I6[3], I6[4]], [I6[3], I6[1], I6[5]], [I6[4], I6[5], I6[2]]])
        ev = np.linalg.eigvalsh(I)
        assert ev.min() > 0 and ev.max() <= ev.sum() - ev.max() + 1e-12  # triangle inequality
    assert list(MODEL["dof_parent"][:6]) == [-1, 0, 1, 2, 3, 4]
    assert len(MODEL["act_dof"]) == 17 and set(MODEL["act_dof"]) == set(range(6, 23))


def test_mass_matrix_matches_jacobian_assembly():
    q, _, _ = _states(3, 1)
    Mc = H.mass_matrix(q)
    h = 1e-6
    fw0 = H.forward(q, np.zeros((3, NV)))
    Mf = np.zeros_like(Mc)
    Jv = np.zeros((3, NB, 3, NV))
    Jw = np.zeros((3, NB, 3, NV))
    for i in range(NV):
        e = np.zeros((3, NV))
        e[:, i] = 1.0
        fp = H.forward(H.advance(q, e, h), np.zeros((3, NV)))
        fm = H.forward(H.advance(q, e, -h), np.zeros((3, NV)))
        for b in range(NB):
            Jv[:, b, :, i] = (np.array(fp["xipos"][b]) - np.array(fm["xipos"][b])).T / (2 * h)
            dR = (np.array(fp["R"][b]) - np.array(fm["R"][b])) / (2 * h)  # [3, 3, E]
            R0 = np.array(fw0["R"][b])
            W = np.einsum("ikE,jkE->Eij", dR, R0)  # dR R0^T = [w]x
            Jw[:, b, :, i] = np.stack([W[:, 2, 1], W[:, 0, 2], W[:, 1, 0]], axis=1)
    for b in range(NB):
        I6 = MODEL["body_inertia"][b]
        Ib = np.array([[I6[0], I6[3], I6[4]], [I6[3], I6[1], I6[5]], [I6[4], I6[5], I6[2]]])
        R0 = np.transpose(np.array(fw0["R"][b]), (2, 0, 1))
        Iw = R0 @ Ib @ np.transpose(R0, (0, 2, 1))
        Mf += MODEL["body_mass"][b] * np.einsum("Eki,Ekj->Eij", Jv[:, b], Jv[:, b])
        Mf += np.einsum("Eki,Ekl,Elj->Eij", Jw[:, b], Iw, Jw[:, b])
    Mf[:, 6:, 6:] += np.diag(MODEL["hinge_arm"])
    np.testing.assert_allclose(Mc, Mf, rtol=1e-6, atol=1e-7 * np.abs(Mc).max())
    assert np.all(np.linalg.eigvalsh(Mc) > 0)
    np.testing.assert_allclose(Mc, np.transpose(Mc, (0, 2, 1)))


def test_free_fall_momentum_theorem():
    """d/dt [L_com; p] = [0; -M g e_z] under any internal forces (no contact at z = 10)."""
    q, qd, rng = _states(4, 2, z=10.0)
    ctrl = rng.uniform(-0.4, 0.4, (4, 17))
    fw = H.forward(q, qd)
    qdd = np.stack(H.accelerations(q, qd, ctrl, fw), axis=1)
    h = 1e-5
    hs = []
    for t in (h, -h):
        fwt = H.forward(H.advance(q, qd, t, qdd), qd + t * qdd)
        hs.append(np.stack(H.spatial_momentum(fwt), axis=1))
    dh = (hs[0] - hs[1]) / (2 * h)
    want = np.zeros_like(dh)
    want[:, 5] = -H.TOTAL_MASS * H.GRAV
    np.testing.assert_allclose(dh, want, atol=2e-4 * H.TOTAL_MASS * H.GRAV)
    # and the contact-free forward carries no external force
    assert all(np.all(np.array(c) == 0) for c in fw["cfrc_ext"])


def _energy(q, qd):
    Mm = H.mass_matrix(q)
    T = 0.5 * np.einsum("Ei,Eij,Ej->E", qd, Mm, qd)
    fw = H.forward(q, qd)
    V = H.TOTAL_MASS * H.GRAV * fw["com"][2] + 0.5 * (MODEL["hinge_stiff"] * q[:, 7:] ** 2).sum(1)
    return T + V


@pytest.mark.parametrize("n_steps", [60])
def test_energy_error_first_order_in_dt(monkeypatch, n_steps):
    """No damping, no limit penalty, no contact: the energy error of the semi-implicit
    Euler step stays bounded (oscillates) and halves with dt."""
    monkeypatch.setitem(MODEL, "hinge_damp", np.zeros(17))
    monkeypatch.setattr(H, "KL", 0.0)
    monkeypatch.setattr(H, "CL", 0.0)
    q0, qd0, _ = _states(2, 3, z=10.0, spread=0.5)
    ctrl = np.zeros((2, 17))
    err = []
    base = H.DT
    for div in (1, 2):  # the same time span at dt and dt / 2
        monkeypatch.setattr(H, "DT", base / div)
        q, qd = q0.copy(), qd0.copy()
        e0 = _energy(q, qd)
        worst = np.zeros(2)
        for k in range(n_steps * div):
            q, qd, _ = H.substep(q, qd, ctrl)
            if (k + 1) % (10 * div) == 0:
                worst = np.maximum(worst, np.abs(_energy(q, qd) - e0))
        err.append(worst)
    assert np.all(err[0] < 1e-3 * e0), (err[0], e0)  # bounded: 0.1 % of the energy
    np.testing.assert_allclose(err[1] / err[0], 0.5, atol=0.1)


def test_random_policy_episode_length_and_rest_on_floor():
    E = 48
    rng = np.random.default_rng(4)
    s = H.humanoid_reset(rng.random((E, H.NU)))
    alive = np.ones(E, bool)
    lens = np.zeros(E, int)
    for t in range(160):
        s, r, d = H.humanoid_step(s, rng.uniform(-0.4, 0.4, (E, 17)))
        lens += alive
        alive &= ~d
        assert np.isfinite(s).all()
    assert 15 <= lens.mean() <= 35, lens.mean()  # MuJoCo Humanoid-v2 under random controls: ~22
    assert not alive.any()
    # fallen and unactuated: comes to rest lying on the floor
    for _ in range(200):
        s, r, d = H.humanoid_step(s, np.zeros((E, 17)))
    q, qd = s[:, :H.NQ], s[:, H.NQ:H.NQ + NV]
    assert np.all(q[:, 2] < 0.4) and np.all(q[:, 2] > 0.03)
    assert np.abs(qd[:, :3]).max() < 0.2
