"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE's own code.

Runs only in the build container (it reads /root/reference, which does not exist
on the GPU box).  The reference cannot be imported whole (Theano/Keras/TF/gym are
absent: ordinary ModuleNotFoundError), so:

* the pure-numpy modules ``misc_utils``, ``running_stat``, ``filters`` and
  ``distributions`` are imported as-is through a stub package whose __path__
  points at /root/reference/modular_rl (bypassing its __init__), and
* ``trpo.cg``, ``trpo.linesearch``, ``trpo.TrpoUpdater.__call__``,
  ``core.compute_advantage``, ``core.add_episode_stats``, ``core.pathlength``,
  ``core.NnVf.fit`` / ``preproc``, ``core.NnRegression.fit`` and
  ``core.LbfgsOptimizer.update`` are AST-extracted from the reference files, with
  the HEAD-only TF diagnostics removed (trpo.py:82,84,98,100,131,132; core.py:79-96),
  and executed; ``ppo.PpoLbfgsUpdater.__call__`` / ``PpoSgdUpdater.__call__`` the same way
  (``python make_golden.py ppo`` writes only ppo_update.npz).

The Theano-compiled callables that ``TrpoUpdater.__call__`` needs
(compute_policy_gradient / compute_losses / compute_fisher_vector_product) and the
VF regression's (predict / f_lossgrad / f_losses, core.py:608,670-671) are injected
from ``oracle/torch_ref.py`` -- torch autograd / double-backward, Theano's own
formulation (trpo.py:29-70, core.py:607-618).  Everything the fixtures record about
CG, step scaling, the line search, the L-BFGS fit and the returned stats is
therefore produced by the reference's own control flow.

Each TRPO / VF case is generated twice: in float64 (truth) and floatX-faithful
(suffix ``f``): the injected graphs evaluate in float32 and ``set_params_flat`` casts
to float32, as Theano with ``floatX=float32`` does (keras_theano_setup.py:5-6,
core.py:540); the reference's numpy code (cg, linesearch, the step scaling) then runs
on the float32 arrays it receives, under this numpy's (2.x) promotion rules.

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
import scipy
import scipy.signal  # noqa: F401  (misc_utils uses scipy.signal via `import scipy`)
import torch

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

    def run_trpo(k, spec, th0, ob, act, adv, oldprob, cfg, dtype):
        """One reference TrpoUpdater.__call__ on a 2-path batch; records under key k."""
        tdt = torch.float64 if dtype == np.float64 else torch.float32
        state = {"th": th0.astype(dtype)}
        self = types.SimpleNamespace(
            cfg=cfg, loss_names=["surr", "kl", "ent"],
            get_params_flat=lambda: state["th"].copy(),
            set_params_flat=lambda t: state.__setitem__("th", np.asarray(t, dtype=dtype).copy()),
            compute_policy_gradient=lambda o, a, ad, op: torch_ref.pg_autograd(spec, state["th"], o, a, ad, op, tdt),
            compute_losses=(lambda o, a, ad, op: list(trpo_np.surr_kl_ent(spec, state["th"], o, a, ad, op)))
            if dtype == np.float64 else (lambda o, a, ad, op: torch_ref.losses(spec, state["th"], o, a, ad, op, tdt)),
            compute_fisher_vector_product=lambda p, o, a, ad, op: torch_ref.fvp_double_backward(
                spec, state["th"], p, o, tdt),
        )
        cast = (lambda a: np.asarray(a).astype(dtype)) if dtype == np.float32 else (lambda a: a)
        N = ob.shape[0]
        paths = [dict(prob=cast(oldprob[:N // 2]), observation=cast(ob[:N // 2]), action=cast(act[:N // 2]),
                      advantage=cast(adv[:N // 2])),
                 dict(prob=cast(oldprob[N // 2:]), observation=cast(ob[N // 2:]), action=cast(act[N // 2:]),
                      advantage=cast(adv[N // 2:]))]
        rec.clear()
        stats = quiet(call, self, paths)
        out[f"{k}_theta1"] = state["th"].astype(np.float64)
        out[f"{k}_stats"] = np.array([stats[n] for n in ("surr_before", "surr_after", "kl_before", "kl_after",
                                                         "ent_before", "ent_after")], dtype=np.float64)
        ls = np.array(rec["ls"], dtype=np.float64)  # rows: (stepfrac, actual, expected, ratio)
        accepted = [i for i, (_, act_i, _, r) in enumerate(ls) if r > 0.1 and act_i > 0]
        for name in ("g", "stepdir", "fullstep"):
            out[f"{k}_{name}"] = np.asarray(rec[name], dtype=np.float64)
        for name in ("shs", "lm", "rate"):
            out[f"{k}_{name}"] = np.float64(rec[name])
        out[f"{k}_ls"] = ls
        out[f"{k}_k"] = np.int64(accepted[0] if accepted else -1)
        # distance of the accept test from its threshold at the accepted backtrack
        out[f"{k}_margin"] = np.float64(ls[accepted[0], 3] - 0.1 if accepted else np.nan)

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
            k = f"{tag}{cfg_i}"
            out[f"{k}_theta0"] = th0
            out[f"{k}_ob"], out[f"{k}_act"], out[f"{k}_adv"], out[f"{k}_oldprob"] = ob, act, adv, oldprob
            out[f"{k}_cfg"] = np.array([cfg["cg_damping"], cfg["max_kl"]])
            run_trpo(k, spec, th0, ob, act, adv, oldprob, cfg, np.float64)
            run_trpo(k + "f", spec, th0, ob, act, adv, oldprob, cfg, np.float32)
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

    # ---------------- TrpoUpdater.__call__ on deep nets (the layered GEMM path): one
    # Dense layer per hid_sizes entry (agentzoo.py:34-36), three hidden layers here
    rng = np.random.default_rng(7)
    out = {}
    for tag, (nin, hid, nout, head, N) in {"deepg": (40, [64, 64, 64], 9, "gauss", 600),
                                           "deepc": (20, [64, 48, 32], 5, "softmax", 500)}.items():
        spec = trpo_np.Spec(nin, hid, nout, head)
        th0 = trpo_np.mlp_init(rng, spec.shapes, head == "gauss")
        th0 = f32(th0 + 0.02 * rng.standard_normal(th0.shape))
        ob = f32(rng.standard_normal((N, nin)))
        oldprob = f32(trpo_np.policy_prob(spec, th0 + 0.01 * rng.standard_normal(th0.shape), ob))
        noise = rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N)
        act = trpo_np.sample(spec, oldprob, noise)
        act = f32(act) if head == "gauss" else act
        adv = f32(trpo_np.standardize(rng.standard_normal(N) + 0.3 * ob[:, 0]))
        for cfg_i, cfg in enumerate([dict(cg_damping=0.1, max_kl=0.01), dict(cg_damping=0.1, max_kl=100.0)]):
            k = f"{tag}{cfg_i}"
            out[f"{k}_theta0"], out[f"{k}_hid"] = th0, np.array(hid)
            out[f"{k}_ob"], out[f"{k}_act"], out[f"{k}_adv"], out[f"{k}_oldprob"] = ob, act, adv, oldprob
            out[f"{k}_cfg"] = np.array([cfg["cg_damping"], cfg["max_kl"]])
            run_trpo(k, spec, th0, ob, act, adv, oldprob, cfg, np.float64)
            run_trpo(k + "f", spec, th0, ob, act, adv, oldprob, cfg, np.float32)
    np.savez(os.path.join(HERE, "trpo_update_deep.npz"), **out)

    # ---------------- NnVf.fit -> NnRegression.fit -> LbfgsOptimizer.update
    # (core.py:652-660, 620-637, 674-697): the reference's own fit, scipy L-BFGS-B with
    # maxiter=2 and mixfrac=0.1 (agentzoo.py:60), on paths of fp32-representable
    # observations and returns; opt_info (funcalls, nit) recorded after core.py:687.
    import scipy.optimize  # noqa: F401  (the extracted update calls scipy.optimize)
    vrec = {}
    ns_v = extract(cr, ["NnVf.fit", "NnVf.preproc", "NnRegression.fit", "LbfgsOptimizer.update"],
                   extra_ns={"np": np, "scipy": scipy, "OrderedDict": OrderedDict, "concat": np.concatenate,
                             "explained_variance_2d": mu.explained_variance_2d, "explained_variance": mu.explained_variance,
                             "_rec": vrec},
                   record_after={687: "_rec.update(funcalls=opt_info['funcalls'], nit=opt_info['nit'])"})
    # NnVf.fit and NnRegression.fit share the name ``fit`` (the later wins in ns_v)
    nnvf_fit = extract(cr, ["NnVf.fit"], extra_ns={"np": np, "concat": np.concatenate})["fit"]
    out = {}
    for tag, (nin, hid, lens, limit, r0) in {"hop": (11, [64, 64], [120, 333, 1, 246], 1000, 3.0),
                                             "cart": (4, [64, 64], [200, 57, 43], 200, 20.0),
                                             "deep": (20, [64, 48, 32], [150, 150, 211], 500, -2.0)}.items():
        spec = trpo_np.Spec(nin + 1, hid, 1, "linear")
        th0 = f32(trpo_np.mlp_init(rng, spec.shapes, False) + 0.05 * rng.standard_normal(spec.P))
        obs = [f32(rng.standard_normal((L, nin))) for L in lens]
        rets = [f32(r0 + 2.0 * rng.standard_normal(L) + np.linspace(0, 1, L)) for L in lens]
        out[f"{tag}_theta0"], out[f"{tag}_hid"], out[f"{tag}_limit"] = th0, np.array(hid), np.int64(limit)
        for i, (o, r) in enumerate(zip(obs, rets)):
            out[f"{tag}_obs{i}"], out[f"{tag}_ret{i}"] = o, r
        out[f"{tag}_npaths"] = np.int64(len(lens))
        for sfx, dtype in (("", np.float64), ("f", np.float32)):
            tdt = torch.float64 if dtype == np.float64 else torch.float32
            state = {"th": th0.astype(dtype)}
            opt = types.SimpleNamespace(
                maxiter=2, all_losses=OrderedDict((n, None) for n in ("loss", "mse", "l2")),
                get_params_flat=lambda: state["th"].copy(),
                set_params_flat=lambda t: state.__setitem__("th", np.asarray(t, dtype=dtype).copy()),
                f_lossgrad=lambda x, y: torch_ref.vf_lossgrad(spec, state["th"], x, y, tdt),
                f_losses=lambda x, y: torch_ref.vf_losses(spec, state["th"], x, y, tdt))
            opt.update = types.MethodType(ns_v["update"], opt)
            reg = types.SimpleNamespace(mixfrac=0.1, opt=opt,
                                        predict=lambda x: torch_ref.vf_predict(spec, state["th"], x, tdt))
            reg.fit = types.MethodType(ns_v["fit"], reg)
            vf = types.SimpleNamespace(reg=reg, timestep_limit=limit)
            vf.preproc = types.MethodType(ns_v["preproc"], vf)
            paths = [dict(observation=o, **{"return": r}) for o, r in zip(obs, rets)]
            vrec.clear()
            # the HEAD NnVf.fit (core.py:652-657) returns (stats, ob_no, vtarg)
            stats, X, vtarg = quiet(nnvf_fit, vf, paths)
            k = tag + sfx
            out[f"{k}_theta1"] = state["th"].astype(np.float64)
            out[f"{k}_stat_keys"] = np.array(list(stats))
            out[f"{k}_stats"] = np.array([float(v) for v in stats.values()], dtype=np.float64)
            out[f"{k}_funcalls"], out[f"{k}_nit"] = np.int64(vrec["funcalls"]), np.int64(vrec["nit"])
            out[f"{k}_X"] = np.asarray(X, dtype=np.float64)
    np.savez(os.path.join(HERE, "vf_fit.npz"), **out)
    ppo_fixtures(mods)
    print("golden fixtures written to", HERE)


def ppo_fixtures(mods):
    """ppo_update.npz: the reference's own PpoLbfgsUpdater.__call__ (ppo.py:59-112) and
    PpoSgdUpdater.__call__ (ppo.py:169-229), AST-extracted, with the Theano functions
    injected from torch autograd (oracle/ppo_np.py: pensurr = surr + kl_coeff kl + 1000
    (kl > 2 kl_target) (kl - cutoff)^2, ppo.py:46-49, 153; adam_updates ppo.py:231-258).
    Each case in float64 and floatX-faithful float32 (suffix f); inputs fp32-representable.
    Recorded: theta after, the returned info, the adapted kl_coeff, scipy's opt_info
    (L-BFGS) and the epoch permutations drawn (SGD, np.random seeded before the call)."""
    from oracle import ppo_np
    import scipy.optimize  # noqa: F401  (the extracted __call__ calls scipy.optimize)
    mu = mods["misc_utils"]
    pp = os.path.join(REF, "ppo.py")
    rec = {}
    base_ns = {"np": np, "scipy": scipy, "OrderedDict": OrderedDict, "concat": np.concatenate,
               "zipsame": mu.zipsame, "fmt_row": mu.fmt_row, "xrange": range, "_rec": rec}
    lb_call = extract(pp, ["PpoLbfgsUpdater.__call__"], extra_ns=dict(base_ns),
                      record_after={90: "_rec.update(funcalls=opt_info['funcalls'], nit=opt_info['nit'], "
                                        "warnflag=opt_info['warnflag'])"})["__call__"]
    # the two epoch-table header prints (ppo.py:185, 190) add a str to a list and raise
    # TypeError in any Python; they are display-only and dropped like the TRPO diagnostics
    sgd_call = extract(pp, ["PpoSgdUpdater.__call__"], drop_lines={185, 190}, extra_ns=dict(base_ns))["__call__"]
    f32 = (lambda a: np.asarray(a, dtype=np.float32).astype(np.float64))
    rng = np.random.default_rng(21)
    out = {}

    def case_inputs(nin, nout, head, N):
        spec = trpo_np.Spec(nin, [64, 64], nout, head)
        th0 = trpo_np.mlp_init(rng, spec.shapes, head == "gauss") + 0.05 * rng.standard_normal(spec.P)
        if head == "gauss":
            th0[-nout:] = -0.3 + 0.1 * rng.standard_normal(nout)
        th0 = f32(th0)
        ob = f32(rng.standard_normal((N, nin)))
        oldprob = f32(trpo_np.policy_prob(spec, th0 + 0.02 * rng.standard_normal(spec.P), ob))
        noise = rng.standard_normal((N, nout)) if head == "gauss" else rng.random(N)
        act = trpo_np.sample(spec, oldprob, noise)
        act = f32(act) if head == "gauss" else act
        adv = f32(trpo_np.standardize(rng.standard_normal(N) + 0.3 * ob[:, 0]))
        return spec, th0, ob, act, adv, oldprob

    info_keys = ["surr_before", "surr_after", "surr_change", "kl_before", "kl_after", "kl_change",
                 "ent_before", "ent_after", "ent_change"]
    test_keys = ["test_" + k for k in info_keys]
    # ---- PpoLbfgsUpdater: (head, N, do_split, reverse_kl, maxiter, kl_coeff0)
    for k, (head, N, split, rev, maxiter, kc0) in {"lbg0": ("gauss", 600, 0, 0, 4, 1.0),
                                                   "lbg1": ("gauss", 600, 1, 1, 4, 0.3),
                                                   "lbc0": ("softmax", 500, 0, 0, 4, 1.0),
                                                   "lbg2": ("gauss", 600, 0, 0, 25, 1.0)}.items():
        nin, nout = (11, 3) if head == "gauss" else (4, 2)
        spec, th0, ob, act, adv, oldprob = case_inputs(nin, nout, head, N)
        out[f"{k}_theta0"], out[f"{k}_ob"], out[f"{k}_act"], out[f"{k}_adv"], out[f"{k}_oldprob"] = \
            th0, ob, act, adv, oldprob
        out[f"{k}_cfg"] = np.array([0.01, maxiter, rev, split, kc0])
        for sfx, dtype in (("", np.float64), ("f", np.float32)):
            tdt = torch.float64 if dtype == np.float64 else torch.float32
            st = {"th": th0.astype(dtype)}
            cfg = mu.update_default_config([("kl_target", float, 1e-2, ""), ("maxiter", int, 25, ""),
                                            ("reverse_kl", int, 0, ""), ("do_split", int, 0, "")],
                                           dict(maxiter=maxiter, reverse_kl=rev, do_split=split))

            def lossgrad(kc, o, a, ad, op, st=st, tdt=tdt):
                l, g = ppo_np.pensurr_and_grad(spec, st["th"], o, a, ad, op, kc, 2 * 0.01, 1000.0, bool(rev), tdt)
                return l, g

            self = types.SimpleNamespace(
                cfg=cfg, kl_coeff=kc0, loss_names=["surr", "kl", "ent"],
                get_params_flat=lambda st=st: st["th"].copy(),
                set_params_flat=lambda t, st=st, dtype=dtype: st.__setitem__("th", np.asarray(t, dtype=dtype).copy()),
                compute_lossgrad=lossgrad,
                compute_losses=lambda o, a, ad, op, st=st, tdt=tdt: ppo_np.losses_t(spec, st["th"], o, a, ad, op,
                                                                                    bool(rev), tdt))
            cast = (lambda a: np.asarray(a).astype(dtype)) if dtype == np.float32 else (lambda a: a)
            h = N // 2
            paths = [dict(prob=cast(oldprob[:h]), observation=cast(ob[:h]), action=cast(act[:h]), advantage=cast(adv[:h])),
                     dict(prob=cast(oldprob[h:]), observation=cast(ob[h:]), action=cast(act[h:]), advantage=cast(adv[h:]))]
            rec.clear()
            info = quiet(lb_call, self, paths)
            kk = k + sfx
            out[f"{kk}_theta1"] = st["th"].astype(np.float64)
            keys = info_keys + (test_keys if split else [])
            out[f"{kk}_info"] = np.array([float(info[n]) for n in keys], dtype=np.float64)
            out[f"{kk}_kl_coeff"] = np.float64(self.kl_coeff)
            out[f"{kk}_funcalls"], out[f"{kk}_nit"] = np.int64(rec["funcalls"]), np.int64(rec["nit"])
    # ---- PpoSgdUpdater: (head, N, do_split, epochs, stepsize, kl_coeff0, seed)
    for k, (head, N, split, epochs, lr, kc0, seed) in {"sgg0": ("gauss", 600, 0, 2, 1e-3, 1.0, 123),
                                                       "sgc0": ("softmax", 600, 0, 2, 1e-3, 1.0, 7),
                                                       "sgg1": ("gauss", 700, 1, 3, 3e-3, 0.3, 99)}.items():
        nin, nout = (11, 3) if head == "gauss" else (4, 3)
        spec, th0, ob, act, adv, _ = case_inputs(nin, nout, head, N)
        out[f"{k}_theta0"], out[f"{k}_ob"], out[f"{k}_act"], out[f"{k}_adv"] = th0, ob, act, adv
        out[f"{k}_cfg"] = np.array([0.01, epochs, lr, split, kc0, seed])
        for sfx, dtype in (("", np.float64), ("f", np.float32)):
            tdt = torch.float64 if dtype == np.float64 else torch.float32
            st = {"th": th0.astype(dtype), "old": None, "m": np.zeros(spec.P, dtype), "v": np.zeros(spec.P, dtype),
                  "t": dtype(0)}
            cfg = mu.update_default_config([("kl_target", float, 1e-2, ""), ("epochs", int, 10, ""),
                                            ("stepsize", float, 1e-3, ""), ("do_split", int, 0, ""),
                                            ("kl_cutoff_coeff", float, 1000.0, "")],
                                           dict(epochs=epochs, stepsize=lr, do_split=split))

            def oldp(o, st=st, tdt=tdt):  # the old net: theta at update_old_net (ppo.py:160, 175)
                return ppo_np.policy_prob_t(spec, st["old"], o, tdt)

            def train(kc, o, a, ad, st=st, tdt=tdt, dtype=dtype, cfg=cfg):
                # outputs at the pre-update params, then the Adam update (ppo.py:155-157, 231-258)
                op = oldp(o)
                l = ppo_np.losses_t(spec, st["th"], o, a, ad, op, False, tdt)
                _, g = ppo_np.pensurr_and_grad(spec, st["th"], o, a, ad, op, kc, 2 * cfg["kl_target"],
                                               cfg["kl_cutoff_coeff"], False, tdt)
                g = g.astype(dtype)
                b1, b2, eps, lr_ = dtype(0.9), dtype(0.999), dtype(1e-8), dtype(cfg["stepsize"])
                st["t"] = st["t"] + dtype(1)
                a_t = lr_ * np.sqrt(dtype(1) - b2 ** st["t"]) / (dtype(1) - b1 ** st["t"])
                st["m"] = b1 * st["m"] + (dtype(1) - b1) * g
                st["v"] = b2 * st["v"] + (dtype(1) - b2) * g ** 2
                st["th"] = (st["th"] - a_t * st["m"] / (np.sqrt(st["v"]) + eps)).astype(dtype)
                return l

            self = types.SimpleNamespace(
                cfg=cfg, kl_coeff=kc0, loss_names=["surr", "kl", "ent"],
                update_old_net=lambda st=st: st.__setitem__("old", st["th"].copy()),
                test=lambda o, a, ad, st=st, tdt=tdt: ppo_np.losses_t(spec, st["th"], o, a, ad, oldp(o), False, tdt),
                train=train)
            cast = (lambda a: np.asarray(a).astype(dtype)) if dtype == np.float32 else (lambda a: a)
            h = N // 2
            paths = [dict(observation=cast(ob[:h]), action=cast(act[:h]), advantage=cast(adv[:h])),
                     dict(observation=cast(ob[h:]), action=cast(act[h:]), advantage=cast(adv[h:]))]
            np.random.seed(seed)
            info = quiet(sgd_call, self, paths)
            kk = k + sfx
            out[f"{kk}_theta1"] = st["th"].astype(np.float64)
            keys = info_keys + (test_keys if split else [])
            out[f"{kk}_info"] = np.array([float(info[n]) for n in keys], dtype=np.float64)
            out[f"{kk}_kl_coeff"] = np.float64(self.kl_coeff)
        train_stop = (int(.75 * N) // 128) * 128 if split else N
        np.random.seed(seed)
        out[f"{k}_perms"] = np.array([np.random.permutation(train_stop) for _ in range(epochs)])
    np.savez(os.path.join(HERE, "ppo_update.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["ppo"]:
        ppo_fixtures(ref_pkg())
    else:
        main()
