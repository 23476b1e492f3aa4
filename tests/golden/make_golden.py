"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE's own code.

Runs only in the build container (it reads /root/reference, which does not exist
on the GPU box).  The reference cannot be imported whole (Theano/Keras/TF/gym are
absent: ordinary ModuleNotFoundError), so:

* the pure-numpy modules ``misc_utils``, ``running_stat``, ``filters`` and
  ``distributions`` are imported as-is through a stub package whose __path__
  points at /root/reference/modular_rl (bypassing its __init__), and
* ``trpo.cg``, ``trpo.linesearch``, ``trpo.TrpoUpdater.__call__``,
  ``core.compute_advantage``, ``core.add_episode_stats`` and ``core.pathlength``
  are AST-extracted from the reference files, with the HEAD-only TF diagnostics
  removed (trpo.py:82,84,98,100,131,132; core.py:79-96), and executed.

The Theano-compiled callables that ``TrpoUpdater.__call__`` needs
(compute_policy_gradient / compute_losses / compute_fisher_vector_product) are
injected from ``oracle/torch_ref.py`` -- torch double-backward, Theano's own
formulation (trpo.py:29-70).  Everything the fixture records about CG, step
scaling, the line search and the returned stats is therefore produced by the
reference's own control flow.

Usage:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
"""
import ast
import contextlib
import io
import os
import sys
import types
from collections import OrderedDict

import numpy as np
import scipy.signal  # noqa: F401  (misc_utils uses scipy.signal via `import scipy`)

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/modular_rl"
sys.path.insert(0, REPO)

from oracle import torch_ref, trpo_np  # noqa: E402


def ref_pkg():
    pkg = types.ModuleType("mrlref")
    pkg.__path__ = [REF]
    sys.modules["mrlref"] = pkg
    import importlib
    mods = {}
    for name in ("misc_utils", "running_stat", "filters", "distributions"):
        mods[name] = importlib.import_module("mrlref." + name)
    return mods


def extract(path, names, drop_lines=(), extra_ns=None, record_after=None):
    """AST-extract top-level defs (or Class.method via 'Class.method') from a reference file.

    ``record_after`` maps a reference line number to a recorder statement (source
    text of this script, not of the reference) appended after that statement, so a
    fixture can keep the reference's own intermediate locals (e.g. shs / lm)."""
    record_after = dict(record_after or {})
    src = open(path).read()
    tree = ast.parse(src)

    def strip(node):
        for field in ("body", "orelse", "finalbody"):
            if hasattr(node, field):
                kept = []
                for st in getattr(node, field):
                    if st.lineno in drop_lines:
                        continue
                    strip(st)
                    kept.append(st)
                    if st.lineno in record_after:
                        kept.extend(ast.parse(record_after[st.lineno]).body)
                if not kept and field == "body":
                    kept = [ast.Pass()]
                setattr(node, field, kept)
        return node

    ns = dict(extra_ns or {})
    for name in names:
        if "." in name:
            cls, meth = name.split(".")
            cnode = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
            fnode = next(n for n in cnode.body if isinstance(n, ast.FunctionDef) and n.name == meth)
        else:
            fnode = next(n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name == name)
        fnode = strip(fnode)
        mod = ast.Module(body=[fnode], type_ignores=[])
        ast.fix_missing_locations(mod)
        exec(compile(mod, path, "exec"), ns)
    return ns


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def main():
    mods = ref_pkg()
    mu = mods["misc_utils"]
    out = {}

    # ---------------- discount (misc_utils.py:9-27) + the a.py:15-23 exactness identity
    rng = np.random.default_rng(1)
    for i, (n, g) in enumerate([(1, 0.99), (7, 0.995), (200, 0.97 * 0.995), (1000, 0.99)]):
        x = rng.standard_normal(n)
        out[f"discount_x{i}"] = x
        out[f"discount_g{i}"] = np.float64(g)
        out[f"discount_y{i}"] = mu.discount(x, g)
    np.savez(os.path.join(HERE, "discount.npz"), **out)

    # ---------------- RunningStat / ZFilter (running_stat.py:4-33, filters.py:17-40)
    out = {}
    RS = mods["running_stat"].RunningStat
    ZF = mods["filters"].ZFilter
    xs = rng.standard_normal((25, 11)) * 3 + 1
    rs = RS((11,))
    zf = ZF((11,), clip=5)
    rf = ZF((), demean=False, clip=10)
    Ms, Ss, vars_, zs, rfs = [], [], [], [], []
    rews = rng.standard_normal(25) + 2
    for t in range(25):
        rs.push(xs[t])
        Ms.append(rs.mean.copy()); Ss.append(rs._S.copy()); vars_.append(rs.var.copy())
        zs.append(zf(xs[t]))
        rfs.append(rf(rews[t]))
    out.update(rs_x=xs, rs_M=np.array(Ms), rs_S=np.array(Ss), rs_var=np.array(vars_),
               zf_out=np.array(zs), rew=rews, rf_out=np.array(rfs), rf_M=rf.rs.mean, rf_S=rf.rs._S, rf_n=rf.rs.n)
    quiet(mods["running_stat"].test_running_stat)  # reference's own unit test passes here
    np.savez(os.path.join(HERE, "filters.npz"), **out)

    # ---------------- categorical_sample (distributions.py:3-13) with the uniforms it drew
    out = {}
    prob = rng.dirichlet(np.ones(3), size=500)
    np.random.seed(123)
    res = mods["distributions"].categorical_sample(prob)
    np.random.seed(123)
    u = np.random.rand(500, 1)[:, 0]
    out.update(prob=prob, u=u, sample=res)
    np.savez(os.path.join(HERE, "categorical_sample.npz"), **out)

    # ---------------- cg / linesearch (trpo.py:143-200)
    tr = os.path.join(REF, "trpo.py")
    ns = extract(tr, ["cg", "linesearch"], extra_ns={"np": np})
    out = {}
    for i, (P, cond) in enumerate([(40, 10.0), (200, 1e3), (5, 1.0)]):
        Q, _ = np.linalg.qr(rng.standard_normal((P, P)))
        A = Q @ np.diag(np.geomspace(1, cond, P)) @ Q.T
        b = rng.standard_normal(P)
        x = quiet(ns["cg"], lambda p: A @ p, b)
        out[f"cg_A{i}"], out[f"cg_b{i}"], out[f"cg_x{i}"] = A, b, x
    # linesearch on a smooth nonconvex function: accept at k=0, k>0, and failure
    c = rng.standard_normal(6)
    f = (lambda th: float(np.sum(np.cos(th) * c) + 0.5 * np.sum(th ** 2)))
    x0 = rng.standard_normal(6)
    gradf = -np.sin(x0) * c + x0
    for i, (scale, rate_mult) in enumerate([(0.05, 1.0), (8.0, 1.0), (0.3, -1.0)]):
        full = -scale * gradf
        rate = rate_mult * float(gradf.dot(gradf)) * scale
        succ, xn = quiet(ns["linesearch"], f, x0, full, rate)
        out[f"ls_full{i}"], out[f"ls_rate{i}"] = full, np.float64(rate)
        out[f"ls_success{i}"], out[f"ls_x{i}"] = np.bool_(succ), xn
    out["ls_xstart"], out["ls_c"] = x0, c
    np.savez(os.path.join(HERE, "cg_linesearch.npz"), **out)

    # ---------------- TrpoUpdater.__call__ (trpo.py:72-140) on small policy batches
    # Every input is fp32-representable (obs, actions, advantages, oldprob, theta0), so
    # the fp32 device pipeline and the float64 reference see identical inputs.  The
    # reference's own locals are recorded: after trpo.py:124 (g, stepdir, shs, lm,
    # fullstep, the expected improve rate) and after trpo.py:154 in linesearch (each
    # backtrack's actual / expected improvement and ratio), so the fixture pins the
    # chosen step size and the accepted backtrack k.
    out = {}
    rec = {}
    ns_tr = extract(tr, ["cg", "linesearch", "TrpoUpdater.__call__"],
                    drop_lines={82, 84, 98, 100, 131, 132},
                    extra_ns={"np": np, "OrderedDict": OrderedDict, "concat": np.concatenate,
                              "zipsame": mu.zipsame, "_rec": rec},
                    record_after={124: "_rec.update(g=g, stepdir=stepdir, shs=shs, lm=lm, fullstep=fullstep, "
                                       "rate=neggdotstepdir / lm)",
                                  154: "_rec.setdefault('ls', []).append((stepfrac, actual_improve, "
                                       "expected_improve, ratio))"})
    call = ns_tr["__call__"]
    f32 = (lambda a: np.asarray(a, dtype=np.float32).astype(np.float64))
    for tag, (nin, nout, head, N) in {"gauss": (11, 3, "gauss", 512), "cat": (4, 2, "softmax", 400)}.items():
        spec = trpo_np.Spec(nin, [64, 64], nout, head)
        th0 = trpo_np.mlp_init(rng, spec.shapes, head == "gauss")
        th0 = f32(th0 + 0.02 * rng.standard_normal(th0.shape))
        ob = f32(rng.standard_normal((N, nin)))
        oldth = th0 + 0.01 * rng.standard_normal(th0.shape)
        oldprob = f32(trpo_np.policy_prob(spec, oldth, ob))
        noise = rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N)
        act = trpo_np.sample(spec, oldprob, noise)
        act = f32(act) if head == "gauss" else act
        adv = f32(trpo_np.standardize(rng.standard_normal(N) + 0.3 * ob[:, 0]))
        # cfg 0: the reference default (rank-deficient for cat: P=4,610 > N=400 rows);
        # cfg 1: the battery settings; cfg 2: a trust region so large the line search backtracks
        for cfg_i, cfg in enumerate([dict(cg_damping=1e-3, max_kl=1e-2), dict(cg_damping=0.1, max_kl=0.01),
                                     dict(cg_damping=0.1, max_kl=100.0)]):
            state = {"th": th0.copy()}
            self = types.SimpleNamespace(
                cfg=cfg, loss_names=["surr", "kl", "ent"],
                get_params_flat=lambda: state["th"].copy(),
                set_params_flat=lambda t: state.__setitem__("th", np.asarray(t, dtype=np.float64).copy()),
                compute_policy_gradient=lambda o, a, ad, op: torch_ref.pg_autograd(spec, state["th"], o, a, ad, op),
                compute_losses=lambda o, a, ad, op: list(trpo_np.surr_kl_ent(spec, state["th"], o, a, ad, op)),
                compute_fisher_vector_product=lambda p, o, a, ad, op: torch_ref.fvp_double_backward(spec, state["th"], p, o),
            )
            paths = [dict(prob=oldprob[:N // 2], observation=ob[:N // 2], action=act[:N // 2], advantage=adv[:N // 2]),
                     dict(prob=oldprob[N // 2:], observation=ob[N // 2:], action=act[N // 2:], advantage=adv[N // 2:])]
            rec.clear()
            stats = quiet(call, self, paths)
            k = f"{tag}{cfg_i}"
            out[f"{k}_theta0"], out[f"{k}_theta1"] = th0, state["th"]
            out[f"{k}_ob"], out[f"{k}_act"], out[f"{k}_adv"], out[f"{k}_oldprob"] = ob, act, adv, oldprob
            out[f"{k}_cfg"] = np.array([cfg["cg_damping"], cfg["max_kl"]])
            out[f"{k}_stats"] = np.array([stats[n] for n in ("surr_before", "surr_after", "kl_before", "kl_after", "ent_before", "ent_after")])
            ls = np.array(rec["ls"], dtype=np.float64)  # rows: (stepfrac, actual, expected, ratio)
            accepted = [i for i, (_, act_i, _, r) in enumerate(ls) if r > 0.1 and act_i > 0]
            out[f"{k}_g"], out[f"{k}_stepdir"], out[f"{k}_fullstep"] = rec["g"], rec["stepdir"], rec["fullstep"]
            out[f"{k}_shs"], out[f"{k}_lm"], out[f"{k}_rate"] = np.float64(rec["shs"]), np.float64(rec["lm"]), np.float64(rec["rate"])
            out[f"{k}_ls"] = ls
            out[f"{k}_k"] = np.int64(accepted[0] if accepted else -1)
            # distance of the accept test from its threshold at the accepted backtrack
            out[f"{k}_margin"] = np.float64(ls[accepted[0], 3] - 0.1 if accepted else np.nan)
    np.savez(os.path.join(HERE, "trpo_update.npz"), **out)

    # ---------------- compute_advantage (core.py:63-105, TF check 79-96 dropped)
    out = {}
    cr = os.path.join(REF, "core.py")
    ns_c = extract(cr, ["compute_advantage", "add_episode_stats", "pathlength"],
                   drop_lines=set(range(79, 97)), extra_ns={"np": np, "discount": mu.discount})
    # set p: five paths (terminated and not) at gamma 0.995, lam 0.97;
    # set q: the same lengths with |mean adv| >> std (rewards around 300, lam 0 so the
    # advantage is the TD residual): an untrained value function's regime, where a
    # single-pass E[x^2]-mean^2 standardisation would cancel (core.py:100-105 is numpy's
    # two-pass std).  Rewards and baselines are fp32-representable.
    f32 = (lambda a: np.asarray(a, dtype=np.float32).astype(np.float64))
    lens = [5, 17, 1, 30, 12]
    for pre, (gam, lam, r0, rs) in {"p": (0.995, 0.97, 1.0, 1.0), "q": (0.995, 0.0, 300.0, 1.0)}.items():
        paths = []
        for i, L in enumerate(lens):
            paths.append(dict(reward=f32(rng.standard_normal(L) * rs + r0), action=np.zeros(L), terminated=(i % 2 == 0),
                              _b=f32(rng.standard_normal(L))))
        vf = types.SimpleNamespace(predict=lambda path: path["_b"])
        quiet(ns_c["compute_advantage"], vf, paths, gam, lam)
        out[f"{pre}_gamma_lam"] = np.array([gam, lam])
        for i, p in enumerate(paths):
            out[f"{pre}{i}_reward"], out[f"{pre}{i}_b"], out[f"{pre}{i}_term"] = p["reward"], p["_b"], np.bool_(p["terminated"])
            out[f"{pre}{i}_adv"], out[f"{pre}{i}_ret"] = p["advantage"], p["return"]
        if pre == "p":
            stats = OrderedDict()
            ns_c["add_episode_stats"](stats, paths)
            out["stats_keys"] = np.array(list(k for k, v in stats.items() if np.ndim(v) == 0))
            out["stats_vals"] = np.array([v for v in stats.values() if np.ndim(v) == 0], dtype=np.float64)
    out["n_paths"] = len(lens)
    np.savez(os.path.join(HERE, "compute_advantage.npz"), **out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
