"""CPU oracle for the modular_rl_amd TRPO hot path -- TEST INFRASTRUCTURE ONLY.

This package is a numpy (float64 by default) restatement of the reference
algorithm in ddlau/modular_rl (`/root/reference`), written from scratch for
this repository.  Every function cites the reference file:line it restates.

Who may import it (and nobody else):
  * ``tests/``                       -- as the parity checker,
  * ``__graft_entry__.smoke()``       -- as the checker of one small invocation,
  * ``bench.py`` ``cpu_baseline`` leg -- timed as the reported CPU baseline.

The product package ``modular_rl_amd`` never imports this; its compute path is
the HIP library ``libmrl_hip.so`` and fails loudly when that is missing.

Pinning (see DESIGN.md "Oracle"):
  * ``discount``, ``RunningStat``/``ZFilter``, ``cg``, ``linesearch``, the
    ``TrpoUpdater.__call__`` control flow and ``compute_advantage`` are pinned
    against the reference's OWN code, AST-extracted and run in the build
    container by ``tests/golden/make_golden.py``; the outputs are committed as
    ``tests/golden/*.npz`` fixtures.
  * The Theano graph (surr/pg/KL/entropy/Fvp, VF loss/grad) cannot run here
    (Theano absent).  It is restated twice -- analytic numpy here and torch
    double-backward (Theano's own formulation, trpo.py:45-58) in
    ``oracle/torch_ref.py`` -- and the two agree to ~1e-15 in float64.
  * Env dynamics (gym CartPole-v0, MuJoCo Hopper-v2) are absent from the
    reference: CartPole is restated from the published gym equations, Hopper-v2
    as articulated rigid-body dynamics of gym's hopper.xml (compliant contact
    instead of MuJoCo's solver), and the Humanoid-shaped env is a surrogate;
    env dynamics are "parity unpinned".
"""
