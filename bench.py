#!/usr/bin/env python
"""Benchmark: full TRPO iterations on Hopper-v2 (articulated-body dynamics), 4096 envs x 1024 steps per GPU.

One "step" = one TRPO iteration of run_policy_gradient_algorithm (core.py:135-171):
lock-step rollout of E x T env steps -> GAE + standardisation -> VF L-BFGS fit ->
TRPO update (pg, 10-iteration CG on the Fisher product, step scaling, line search).
Inputs are synthetic (random-init nets, simulator-generated data); all device work
starts from state already resident in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  value = env-steps/s summed over ranks (weak scaling:
E x T envs-steps per GPU per iteration).  Also reported: TRPO-iters/s, per-phase
times, the live HIP-event roofline of the dominant kernel (by device time per iteration:
the persistent rollout on C3) and of the GAE scan, and the CPU oracle timed on a bounded
sample of the workload.  Defaults: N = 1, K = 20, W = 5 (well under a minute of GPU time).
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec + TRPO-iters/sec, 4096 envs×1024 steps, 1/2/4/8 MI355X"
PEAK_FP32_TFLOPS = 157.3     # MI355X dense FP32 (MFMA f32 == VALU rate), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2500.0    # MI355X dense BF16 MFMA (no 2:1 sparsity), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec


def flops_per_row(net):
    """Algorithmic FLOP per row of the two timed halves of the Fisher product.
    The primal forward of the update's theta is cached (fused net: h1/h2 activation
    cache; layered net: the recorded tape), so fvp_jvp_rows = JVP only (layer 0 one
    product, deeper layers two) and fvp_vjp = weight grads of every layer + input grads
    of layers >= 1.  Without the cache the fused JVP kernel also recomputes the forward."""
    dims = [net.n_in] + list(net.hid_sizes) + [net.n_out]
    mm = [dims[i] * dims[i + 1] for i in range(len(dims) - 1)]
    jvp = 2 * (mm[0] + 2 * sum(mm[1:]))
    vjp = 2 * (sum(mm) + sum(mm[1:]))
    fwd = 2 * sum(mm)
    if getattr(net, "layered", False) or getattr(net, "use_cache", False):
        # the primal forward comes from the activation cache / recorded tape
        return {"fvp_jvp_rows": jvp, "fvp_vjp": vjp, "fvp_onepass": jvp + vjp, "policy_forward": fwd}
    return {"fvp_jvp_rows": fwd + jvp, "fvp_vjp": vjp, "fvp_onepass": fwd + jvp + vjp, "policy_forward": fwd}


def vjp_binary_entry(kern, policy_vjp_flop, vf_vjp_flop, rows, iters):
    """One entry for the VJP kernel binary over its timed roles -- the Fisher products
    (fvp_vjp), the policy gradient (pg_vjp) and the VF fit evaluations (vf_vjp) --
    as rocprofv3 sums one kernel name: launches, summed HIP-event time, mean per
    launch and the launch-weighted algorithmic FLOP per row.  ``kern`` maps a role to
    (launches, mean_ms, total_ms); None without Fisher-product launches."""
    roles = {"fvp_vjp": policy_vjp_flop, "pg_vjp": policy_vjp_flop, "vf_vjp": vf_vjp_flop}
    parts = {r: kern[r] for r in roles if r in kern and roles[r] is not None}
    if "fvp_vjp" not in parts:
        return None
    cnt = sum(c for c, _, _ in parts.values())
    tot = sum(t for _, _, t in parts.values())
    flop = sum(c * roles[r] * rows for r, (c, _, _) in parts.items())
    return dict(launches=cnt, mean_ms=tot / cnt, total_ms=tot, rows_per_launch=rows, flop_per_row=flop / (cnt * rows),
                roles={r: {"launches": c, "mean_ms": round(m, 5), "ms_per_iter": round(t / iters, 3)}
                       for r, (c, m, t) in parts.items()})


VJP_BINARY = {"fp32": "mlp_vjp16_kernel", "bf16": "mlp_vjp_bf16_kernel"}  # the cached VJP per dtype


def dominant_kernel(kinfo):
    """The kernel binary with the largest device time per iteration (fvp_vjp is one
    role of the VJP binary when that entry exists)."""
    vjp = [k for k in kinfo if k in VJP_BINARY.values()]
    cands = [k for k in kinfo if not (k == "fvp_vjp" and vjp)]
    return max(cands, key=lambda k: kinfo[k]["total_ms"])


DYNAMICS = {"Hopper-v2": "hopper.xml articulated-body dynamics", "Humanoid-v2": "humanoid.xml articulated-body dynamics",
            "CartPole-v0": "gym equations"}
GAE_BYTES_PER_ROW = 17  # read r 4 + v 4 + flags 1, write adv 4 + ret 4
PMC_FILE = "pmc_r06.json"  # tools/evidence.sh pmc (FETCH_SIZE x2 + WRITE_SIZE per launch, separate passes)
GEMM_PMC_FILE = "pmc_gemm_r04.json"  # tools/pmc_traffic.py --gemm: HBM bytes per layered GEMM launch
# SQ issue cycles per rollout step (tools/rollout_issue.py: persistent kernel; tools/step_issue.py: the
# layered Humanoid step's launch chain), newest first: the first file holding the line's key is used
ROLLOUT_ISSUE_FILES = ("rollout_issue_r06.json", "rollout_issue_r05.json", "rollout_issue_r04.json", "rollout_issue_r03.json")
CLOCK_GHZ = 2.4  # MI355X max shader clock (MI355X_MICROARCH.md)


def host_info():
    """The box the CPU baseline ran on: logical CPUs, the affinity set this
    process may use, the CPU model, and the torch / BLAS thread counts."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        from threadpoolctl import threadpool_info
        blas = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        blas = None
    aff = os.sched_getaffinity(0)
    cores = set()
    for c in aff:  # physical cores of the affinity set (SMT siblings share one)
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                cores.add(f.read().strip())
        except OSError:
            cores.add(str(c))
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": len(aff), "affinity_physical_cores": len(cores),
            "cpu_model": model, "torch_threads": torch.get_num_threads(), "blas_threads": blas,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "threads_note": "the GPU box gives each one-GPU job a 16-CPU share of the host (OMP_NUM_THREADS=16, set "
                            "by the harness, which asks jobs to keep their pools to that share); the affinity set "
                            "lists the whole host, so the baseline uses the share, not every physical core"}


def cpu_serial_c1(seconds=8.0, seed=0):
    """the reference's serial loop restated -- ONE
    CartPole env, a single-row (M = 1) policy forward per step (core.py:182-221,
    StochPolicy.act core.py:261-267), then GAE, the VF fit and the TRPO update on the
    batch (timesteps_per_batch 200, whole episodes: core.py:210-221).  Iterations
    repeat until ``seconds`` have passed; one core (numpy per-row work)."""
    from oracle import rollout_np as RO
    from oracle import trpo_np as T
    rng = np.random.default_rng(seed)
    spec = T.Spec(4, [64, 64], 2, "softmax")
    vspec = T.Spec(5, [64, 64], 1, "linear")
    th = T.mlp_init(rng, spec.shapes, False)
    thv = T.mlp_init(rng, vspec.shapes, False)
    fs = RO.FilterState(5)
    steps = iters = 0
    from threadpoolctl import threadpool_limits
    limit = threadpool_limits(1)  # one core, like the reference's single process
    torch_threads = torch.get_num_threads()
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        envs = RO.Envs(RO.CARTPOLE, 1, seed + iters)
        out, fs = RO.collect(envs, fs, spec, th, 200, 200, iters)  # E = 1: one row per step
        N = 200
        ob = out["obs"].reshape(N, 4).astype(np.float64)
        X = np.concatenate([ob, (out["ep_t"].reshape(N) / 200.0)[:, None]], axis=1)
        v = T.mlp_forward(vspec, thv, X, np.float32)[0][:, 0].astype(np.float64).reshape(200, 1)
        flags = out["flags"]
        adv, ret = T.gae_batched(out["rew"].astype(np.float64), v, (flags & 1) > 0, (flags & 2) > 0, 0.995, 0.97)
        adv = T.standardize(adv).reshape(N)
        thv, _, _, _ = T.vf_fit(vspec, thv, X, ret.reshape(N), mixfrac=0.1, maxiter=2, dtype=np.float32)
        act = out["act"].reshape(N, -1).astype(np.float64)[:, 0]
        th, _, _ = T.trpo_update(spec, th, ob, act, adv, out["prob"].reshape(N, -1).astype(np.float64),
                                 cg_damping=0.1, max_kl=0.01, dtype=np.float32)
        steps += N
        iters += 1
    dt = time.perf_counter() - t0
    limit.unregister()
    torch.set_num_threads(torch_threads)
    return {"value": steps / dt, "unit": "env-steps/s", "trpo_iters_per_sec": iters / dt, "cores": 1, "kind": "port",
            "box": host_info(),
            "sample": f"C1: {iters} serial TRPO iterations of ONE CartPole-v0 env x 200 steps, one-row policy forward "
                      f"per step, numpy oracle, {dt:.1f} s"}


def cpu_baseline(E, Tn, env_id="Hopper-v2", hid=(64, 64), seed=0):
    """Time the numpy oracle (CPU restatement of the reference) on one full iteration."""
    from oracle import fma
    from oracle import rollout_np as RO
    from oracle import trpo_np as T
    box = host_info()
    # threads the numpy / BLAS work can actually run on: the BLAS pool, within the affinity set
    threads = min(box["blas_threads"] or box["affinity_cpus"], box["affinity_cpus"])
    rng = np.random.default_rng(seed)
    kind, O, A, limit = {"Hopper-v2": (RO.HOPPER, 11, 3, 1000), "Humanoid-v2": (RO.HUMANOID, 376, 17, 1000),
                         "CartPole-v0": (RO.CARTPOLE, 4, 2, 200)}[env_id]
    head = "softmax" if env_id == "CartPole-v0" else "gauss"
    spec = T.Spec(O, list(hid), A, head)
    vspec = T.Spec(O + 1, list(hid), 1, "linear")
    th = T.mlp_init(rng, spec.shapes, head == "gauss")
    thv = T.mlp_init(rng, vspec.shapes, False)
    envs = RO.Envs(kind, E, seed)
    fs = RO.FilterState(O + 1)
    t0 = time.perf_counter()
    with fma.plain():  # multiply-adds as a*b + c: the exact fma emulation is for parity only
        out, fs = RO.collect(envs, fs, spec, th, Tn, limit, 0)
    N = E * Tn
    ob = out["obs"].reshape(N, O).astype(np.float64)
    X = np.concatenate([ob, (out["ep_t"].reshape(N) / float(limit))[:, None]], axis=1)
    v = T.mlp_forward(vspec, thv, X, np.float32)[0][:, 0].astype(np.float64).reshape(Tn, E)
    flags = out["flags"]
    adv, ret = T.gae_batched(out["rew"].astype(np.float64), v, (flags & 1) > 0, (flags & 2) > 0, 0.995, 0.97)
    adv = T.standardize(adv).reshape(N)
    T.vf_fit(vspec, thv, X, ret.reshape(N), mixfrac=0.1, maxiter=2, dtype=np.float32)
    act = out["act"].reshape(N, -1).astype(np.float64)
    T.trpo_update(spec, th, ob, act[:, 0] if head == "softmax" else act, adv,
                  out["prob"].reshape(N, -1).astype(np.float64), cg_damping=0.1, max_kl=0.01, dtype=np.float32)
    dt = time.perf_counter() - t0
    return {"value": N / dt, "unit": "env-steps/s", "cores": int(threads), "kind": "port", "box": box,
            "sample": f"one full TRPO iteration (rollout+GAE+VF fit+update) of the numpy oracle on {env_id} "
                      f"{E} envs x {Tn} steps = {N} env-steps, net {O}-{'-'.join(map(str, hid))}-{A}, "
                      f"float32 update / float64 rollout (multiply-adds unfused), {dt:.1f} s"}


def rollout_latency_roofline(ki, key, pmc, K, layered=False):
    """The rollout step is a latency chain (one wave per SIMD, a cross-block hand-off per
    step), bound by neither MFMA nor HBM: its roof is the wave's own instruction issue
    time per step (SQ_ACTIVE_INST_ANY per wave per step from a committed PMC pass,
    tools/rollout_issue.py) at the 2.4 GHz clock.  achieved = the live step time,
    frac = issue floor / achieved."""
    us = ki["mean_ms"] * 1e3
    issue, src = {}, None
    for fn in ROLLOUT_ISSUE_FILES:
        path = os.path.join(ROOT, "profiles", fn)
        if os.path.exists(path):
            with open(path) as f:
                issue = json.load(f).get(key, {})
            if issue:
                src = fn
                break
    floor = issue["issue_cycles_per_step"] / (CLOCK_GHZ * 1e3) if issue else None
    out = {"bound": "latency", "achieved": round(us, 3), "peak": round(floor, 3) if floor else None, "unit": "us/step",
           "frac": round(floor / us, 4) if floor else None,
           "traffic": pmc.get("rollout_step", {}).get("hbm_bytes_per_launch"),
           "kernel": "rollout_persistent_kernel (per step)", "cycles_per_step_at_2.4GHz": round(us * CLOCK_GHZ * 1e3),
           "issue_cycles_per_step": round(issue["issue_cycles_per_step"]) if issue else None,
           "valu_insts_per_step": round(issue["valu_insts_per_step"]) if issue else None,
           "issue_source": f"profiles/{src}[{key}] (rocprofv3 SQ pass)" if issue else None,
           "mean_launch_ms": round(ki["mean_ms"], 5), "launches_timed": ki["launches"],
           "ms_per_iter": round(ki["total_ms"] / K, 3),
           "mfma_frac_of_forward": round(ki["frac_mfma"], 5),
           "note": ("latency-bound: one persistent launch runs the T steps, each a filter merge over all envs "
                    "(cross-block hand-off) + the policy forward + fp64 env substeps, one wave per SIMD on E/64 CUs; "
                    "peak = the wave's instruction-issue time per step (PMC), achieved = rollout region / T")}
    if layered:
        # the layered (Humanoid) rollout is a chain of launches per step, no persistent kernel
        out["kernel"] = ("layered rollout step (lrollout_obs, the hidden-layer GEMMs, hm_act_kernel: fused head + "
                         "wave-per-env fp64 dynamics, lrollout_partials)")
        out["note"] = ("latency-bound: per step a filter-merge launch, the policy's hidden layers as GEMMs over the "
                       "E rows, and the env step with one wave per env (hm_act_kernel, the largest part); peak = the "
                       "sum over the step's launches of one wave's instruction-issue time (SQ pass over the rollout, "
                       "tools/step_issue.py); achieved = rollout region / T")
        if issue.get("kernels"):
            out["issue_per_kernel_us"] = {k: round(v["per_step"] * v["issue_cycles_per_wave"] / (CLOCK_GHZ * 1e3), 3)
                                          for k, v in issue["kernels"].items()}
    return out


def fisher_arith(net):
    """How the line's Fisher-vector products multiply (config.fisher_product)."""
    if getattr(net, "layered", False) or getattr(net, "bf16", False):
        return "as the MLP dtype"
    jvp = "split-operand bf16 MFMA (fp32 operands split exactly into 3 bf16 parts, f32 accumulate)" \
        if getattr(net, "fisher_split", False) else "exact f32 MFMA"
    vjp = ("hybrid: the two 64x64 products of each 16-row tile (gh1, gW1) on split-operand bf16 MFMA, "
           "the rest exact f32 MFMA (mlp_vjp16_kernel<HYB>)")
    if getattr(net, "fisher_onepass", False):
        return {"pass": "one kernel per product (mlp_fisher_hyb_kernel: per block 4 waves of JVP rows + KL metric "
                        "and 4 waves of the hybrid VJP, the head rows through LDS)", "jvp_rows": jvp, "vjp": vjp}
    return {"pass": "two kernels per product (JVP + metric rows, then the VJP)", "jvp_rows": jvp, "vjp": vjp}


def gae_back_to_back(batch, cfg, reps=20):
    """ms per mrl_gae launch, `reps` launches back to back on `batch` (its adv / ret rows are
    rewritten with the same values), one event pair on the launch stream."""
    from modular_rl_amd.core import gae_scan
    s = torch.cuda.current_stream()
    gae_scan(batch, cfg["gamma"], cfg["lam"])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        gae_scan(batch, cfg["gamma"], cfg["lam"])
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def policy_gemm_roofline(kern, kinfo, net, dtype, n_rows, K, pmc, gemm_pmc):
    """north_star's "MFMA roofline for the policy GEMM" (agentzoo.py:34-37 Dense layers):
    the policy MLP's largest GEMM binary by device time per iteration -- on the fused
    64-wide path the Fisher-product kernels (each a whole forward-mode / reverse-mode MLP
    pass of K = 64 GEMMs on MFMA), on the layered path the largest of the individually
    timed GEMM launches -- its algorithmic FLOP / mean HIP-event launch time / the dtype's
    dense MFMA peak, and the PMC traffic / algorithmic bytes ratio where a pass measured it."""
    peak = PEAK_BF16_TFLOPS if dtype == "bf16" else PEAK_FP32_TFLOPS
    if not net.layered:
        cands = {k: v for k, v in kinfo.items()
                 if k in ("fvp_onepass", "fvp_jvp_rows") + tuple(VJP_BINARY.values())}
        if not cands:
            return None
        name = max(cands, key=lambda k: cands[k]["total_ms"])
        ki = cands[name]
        role = "fvp_vjp" if name in VJP_BINARY.values() else name
        alg = ki.get("bytes_per_row", 0) * ki["rows_per_launch"]
        traffic = pmc.get(role, {}).get("hbm_bytes_per_launch")
        return {"bound": "mfma", "achieved": round(ki["tflops"], 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ki["tflops"] / peak, 4), "traffic": traffic,
                "traffic_over_algorithmic": round(traffic / alg, 3) if traffic and alg else None,
                "algorithmic_bytes": alg or None,
                "kernel": {"fvp_jvp_rows": ("mlp_fvp_split_kernel (JVP + KL metric)"
                                            if getattr(net, "fisher_split", False)
                                            else "mlp_rows_kernel (JVP + KL metric)"),
                           "fvp_onepass": "mlp_fisher_hyb_kernel (JVP + KL metric + hybrid VJP, one launch)"
                           }.get(name, name),
                "flop_per_row": ki["flop_per_row"], "rows_per_launch": ki["rows_per_launch"],
                "mean_launch_ms": round(ki["mean_ms"], 5), "launches_timed": ki["launches"],
                "ms_per_iter": round(ki["total_ms"] / K, 3),
                "note": "fused 64-wide policy MLP: each Fisher-product / gradient pass is one kernel whose GEMMs "
                        "(K = 64 hidden units, N = rows) run on MFMA; achieved = its algorithmic FLOP / HIP-event time"}
    from modular_rl_amd import timing
    g = {k: v for k, v in kern.items() if k.startswith("gemm:")}
    if not g:
        return None
    name = max(g, key=lambda k: g[k][2])
    cnt, mean_ms, tot_ms = g[name]
    m = timing.meta.get(name, {})
    tf = m["flop"] / (mean_ms * 1e-3) / 1e12
    gemm_peak = PEAK_BF16_TFLOPS if m.get("dtype") == "bf16" else PEAK_FP32_TFLOPS
    split = m.get("dtype") == "split"
    if split:
        # fp32 on split operands: six bf16 part products per fp32 product on the bf16 MFMA,
        # so the MFMA work is 6x the algorithmic FLOP, priced against the bf16 peak
        tf, gemm_peak = 6 * tf, PEAK_BF16_TFLOPS
    traffic = gemm_pmc.get(name, {}).get("hbm_bytes_per_launch") if gemm_pmc else None
    by_shape = {k: {"launches": c, "mean_ms": round(mm, 4), "ms_per_iter": round(t / K, 3),
                    "frac_mfma": round(timing.meta[k]["flop"] / (mm * 1e-3) / 1e12 *
                                       (6 if timing.meta[k].get("dtype") == "split" else 1) /
                                       (PEAK_BF16_TFLOPS if timing.meta[k].get("dtype") in ("bf16", "split")
                                        else PEAK_FP32_TFLOPS), 4)}
                for k, (c, mm, t) in sorted(g.items(), key=lambda kv: -kv[1][2])}
    return {"bound": "mfma", "achieved": round(tf, 3), "peak": gemm_peak, "unit": "TFLOP/s",
            "frac": round(tf / gemm_peak, 4), "traffic": traffic,
            "traffic_over_algorithmic": round(traffic / m["bytes"], 3) if traffic else None,
            "traffic_source": f"profiles/{GEMM_PMC_FILE} (PMC, separate passes)" if traffic else None,
            "algorithmic_bytes": m["bytes"], "hbm_gbs_alg": round(m["bytes"] / (mean_ms * 1e-3) / 1e9, 1),
            "kernel": f"{m.get('kernel')} {name}", "flop_per_launch": m["flop"],
            "mean_launch_ms": round(mean_ms, 5), "launches_timed": cnt, "ms_per_iter": round(tot_ms / K, 3),
            "gemms": by_shape,
            "note": "layered path: every GEMM launch over >= 65,536 rows timed on its own (HIP events on its stream); "
                    "the shape with the largest device time per iteration; flop = 2mnk per product"
                    + ("; fp32 on split bf16 operands: achieved = 6 x 2mnk / time (the six part products on bf16 "
                       "MFMA) against the bf16 peak" if split else "")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 20 timed iterations after 5 warmup ones (the last VF fit's drain, timed as
    # part of iteration K, amortised over 20; the per-launch timing samples 5 of them)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--env", default="Hopper-v2")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=1024)
    ap.add_argument("--hid", default=None, help="hidden sizes, e.g. 512,512,512 (default 64,64; Humanoid 512x3)")
    ap.add_argument("--cpu-envs", type=int, default=None)
    ap.add_argument("--cpu-horizon", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="MFMA operand precision of every MLP pass (fp32: the parity dtype; bf16: throughput mode)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run the VF fit in the reference order instead of beside the next rollout")
    args = ap.parse_args()
    # stdout carries exactly the one JSON line: whatever else reaches file descriptor 1 --
    # native libraries' banners (RCCL prints its version block there when a communicator
    # is created) or a stray print -- is sent to stderr, and the line goes to a duplicate
    # of the original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    from modular_rl_amd import timing
    from modular_rl_amd.agentzoo import TrpoAgent
    from modular_rl_amd.core import IterationRunner
    from modular_rl_amd.dist import init_from_env
    from modular_rl_amd.envs import make

    comm = init_from_env()
    if torch.cuda.is_available() and not comm.enabled:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    rank, world = comm.rank, comm.world
    env = make(args.env)
    E, Tn = args.envs, args.horizon
    humanoid = args.env == "Humanoid-v2"
    hid = [int(h) for h in args.hid.split(",")] if args.hid else ([512, 512, 512] if humanoid else [64, 64])
    cpu_E = args.cpu_envs or (64 if humanoid else 1024)
    cpu_T = args.cpu_horizon or (64 if humanoid else 256)
    cfg = dict(timestep_limit=env.spec.max_episode_steps, gamma=0.995, lam=0.97, max_kl=0.01, cg_damping=0.1,
               n_envs=E, horizon=Tn, filter=1, seed=0, hid_sizes=hid, activation="tanh", use_graph=1,
               mlp_dtype=args.dtype)
    agent = TrpoAgent(env.observation_space, env.action_space, cfg, comm=comm)
    collector = agent.make_collector(env, cfg)
    runner = IterationRunner(agent, collector, cfg, comm, pipeline=not args.no_pipeline)

    phases = {"rollout": 0.0, "advantage": 0.0, "vf_fit": 0.0, "trpo_update": 0.0}
    spans = {"rollout": ("rollout0", "rollout1"), "advantage": ("adv0", "adv1"), "vf_fit": ("vf0", "vf1"),
             "trpo_update": ("upd0", "upd1")}
    recs = []

    with runner.loop_stream():  # no legacy-stream operations between the steps (IterationRunner.loop_stream)
        for i in range(args.warmup):
            runner.step(prelaunch_next=i + 1 < args.warmup)
        runner.drain()
    # the per-launch regions (Fisher products, VJPs, GEMMs, the GAE scan) and the phase
    # spans are recorded on every 4th timed iteration only (each event is a queue marker
    # that delays the next kernel); their per-iteration figures are the sampled
    # iterations' means, scaled to K (modular_rl_amd/timing.py).  The rollout region is
    # recorded on every iteration.
    timing.enable(True, detail_every=4)
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # K whole iterations: K rollouts, advantages, VF fits and policy updates (the last
    # VF fit drains inside the timed region)
    with runner.loop_stream():
        for i in range(args.steps):
            timing.tick()
            runner.step(prelaunch_next=i + 1 < args.steps)  # the next rollout issued as theta is final
            recs.append(runner.last_phase_events)
        runner.drain()
    recs.append(runner.last_drain_events if runner.pipeline else {})
    torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    if comm.enabled:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    kern = timing.summary()
    timing.enable(False)
    nph = {k: 0 for k in phases}
    for ev in recs:
        for k, (a, b) in spans.items():
            # (the first timed iteration's rollout was issued in the warmup, untimed)
            if ev.get(a) is not None and ev.get(b) is not None:
                phases[k] += ev[a].elapsed_time(ev[b])
                nph[k] += 1
    # per-iteration phase times over the iterations that timed them, scaled to K
    phases = {k: (v / nph[k] * args.steps if nph[k] else 0.0) for k, v in phases.items()}
    K = args.steps
    n_local = E * Tn
    total_steps = n_local * world * K
    value = total_steps / elapsed
    if rank != 0:
        return runner
    fpr = flops_per_row(agent.policy.net)
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_FP32_TFLOPS
    net = agent.policy.net
    # algorithmic HBM bytes per row of the fused Fisher-product kernels: the primal
    # activation cache (h1 + h2: 512 B fp32, 256 B bf16), the obs row, the head rows
    cache_b = 0 if net.layered else (256 if args.dtype == "bf16" else 512)
    row_b = cache_b + 4 * net.n_in + 4 * net.gh
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", PMC_FILE)  # measured on the default Hopper config
    if (os.path.exists(pmc_path) and args.env == "Hopper-v2" and not agent.policy.net.layered and E == 4096
            and Tn == 1024 and args.dtype == "fp32"):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if "fvp_jvp_rows" not in pmc and "fvp_jvp_rows_split" in pmc:  # the JVP half's kernel this round
            pmc["fvp_jvp_rows"] = pmc["fvp_jvp_rows_split"]
    kinfo = {}
    for name in ("fvp_onepass", "fvp_jvp_rows", "fvp_vjp"):
        if name in kern:
            cnt, mean_ms, tot_ms = kern[name]
            kinfo[name] = dict(launches=cnt, mean_ms=mean_ms, total_ms=tot_ms, rows_per_launch=n_local,
                               flop_per_row=fpr[name])
            if not net.layered:
                # one pass: the cache and the obs row cross HBM, the head rows stay in LDS
                rb = cache_b + 4 * net.n_in if name == "fvp_onepass" else row_b
                kinfo[name]["bytes_per_row"] = rb
                kinfo[name]["hbm_gbs_alg"] = rb * n_local / (mean_ms * 1e-3) / 1e9
    if not net.layered:
        # the same kernel binary (the cached VJP) also serves the policy gradient and every
        # VF L-BFGS evaluation (the VF fit's launches run beside the next rollout on the
        # fit's CU set): rocprofv3 sums them into one entry, so the dominance test does too
        vf_net = agent.baseline.net
        vjp = vjp_binary_entry(kern, fpr["fvp_vjp"], None if vf_net.layered else flops_per_row(vf_net)["fvp_vjp"],
                               n_local, K)
        if vjp is not None:
            vjp["bytes_per_row"] = row_b  # the Fisher-product launch's algorithmic bytes (PMC: the same)
            kinfo[VJP_BINARY[args.dtype]] = vjp
    if "rollout_steps" in kern:
        # one timed region per iteration around the rollout's launches (the persistent
        # kernel over the T steps, in a graph on the rollout stream): region / T per step
        cnt, mean_ms, tot_ms = kern["rollout_steps"]
        kinfo["rollout_step"] = dict(launches=cnt * Tn, mean_ms=mean_ms / Tn, total_ms=tot_ms, rows_per_launch=E,
                                     flop_per_row=fpr["policy_forward"], step_to_step=True)
    for name, ki in kinfo.items():
        ki["tflops"] = ki["flop_per_row"] * ki["rows_per_launch"] / (ki["mean_ms"] * 1e-3) / 1e12
        ki["frac_mfma"] = ki["tflops"] / peak
        if pmc.get(name, {}).get("hbm_bytes_per_launch"):
            ki["hbm_gbs_pmc"] = pmc[name]["hbm_bytes_per_launch"] / (ki["mean_ms"] * 1e-3) / 1e9
    dom = dominant_kernel(kinfo)
    is_vjp = dom in VJP_BINARY.values()
    traffic = pmc.get("fvp_vjp" if is_vjp else dom, {}).get("hbm_bytes_per_launch")
    roofline = {"bound": "mfma", "achieved": round(kinfo[dom]["tflops"], 3), "peak": peak,
                "unit": "TFLOP/s", "frac": round(kinfo[dom]["tflops"] / peak, 4), "traffic": traffic,
                "traffic_source": f"profiles/{PMC_FILE} (PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes; "
                                  "not measured in this run)" if traffic else None,
                "kernel": dom, "flop_per_row": kinfo[dom]["flop_per_row"],
                "rows_per_launch": kinfo[dom]["rows_per_launch"],
                "mean_launch_ms": round(kinfo[dom]["mean_ms"], 5), "launches_timed": kinfo[dom]["launches"],
                "ms_per_iter": round(kinfo[dom]["total_ms"] / K, 3)}
    if is_vjp:
        roofline["roles"] = kinfo[dom]["roles"]
        roofline["note"] = ("all launches of the VJP kernel binary (Fisher products, policy gradient, VF fit "
                            "evaluations); achieved = their algorithmic FLOP / their summed HIP-event durations; "
                            "traffic: the Fisher-product launch's PMC bytes")
    if dom == "rollout_step":
        roofline = rollout_latency_roofline(kinfo[dom], f"{args.env}/{args.dtype}", pmc, K, layered=net.layered)
    gemm_pmc = {}
    gp = os.path.join(ROOT, "profiles", GEMM_PMC_FILE)
    if os.path.exists(gp) and net.layered:
        with open(gp) as f:
            gemm_pmc = json.load(f).get(f"{args.env}/{args.dtype}/{E}", {})
    pg_roof = policy_gemm_roofline(kern, kinfo, net, args.dtype, n_local, K, pmc, gemm_pmc)
    gae = None
    if "gae_scan" in kern:
        cnt, mean_ms, _ = kern["gae_scan"]
        # the scan launched back to back on the last iteration's batch, one HIP event pair
        # around 20 launches on its stream: the kernel's own duration (the in-loop region
        # also holds its two event markers, ~10 us of queue latency around a ~15 us kernel)
        b2b_ms = gae_back_to_back(runner.last_batch, cfg)
        gbs = GAE_BYTES_PER_ROW * n_local / (b2b_ms * 1e-3) / 1e9
        gae = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
               "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": pmc.get("gae_scan", {}).get("hbm_bytes_per_launch"),
               "bytes_per_row": GAE_BYTES_PER_ROW, "mean_launch_ms": round(b2b_ms, 4),
               "mean_launch_ms_in_loop": round(mean_ms, 4),
               "note": "achieved / mean_launch_ms: mrl_gae x 20 back to back on the bench's last batch after the "
                       "timed region (HIP events on its stream); mean_launch_ms_in_loop: the in-loop region "
                       "(sampled iterations), which includes its event markers' queue latency"}
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1000, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
        "config": {"workload": f"{args.env} ({DYNAMICS[args.env]}) {E} envs x {Tn} steps per GPU, one TRPO iteration "
                               "per step (rollout+GAE+VF L-BFGS+TRPO CG/linesearch)",
                   "envs_per_gpu": E, "horizon": Tn, "global_batch": E * Tn * world, "parallelism": f"dp{world}",
                   "policy": f"{env.obs_dim}-{'-'.join(map(str, hid))}-{env.act_dim} tanh "
                             f"{'Categorical' if args.env == 'CartPole-v0' else 'DiagGauss'} "
                             f"({'layered GEMM' if agent.policy.net.layered else 'fused'} path)",
                   "mlp_dtype": args.dtype, "gamma": 0.995, "lam": 0.97,
                   "max_kl": 0.01, "cg_damping": 0.1,
                   "vf_fit_beside_next_rollout": runner.pipeline,
                   "fisher_product": fisher_arith(agent.policy.net)},
        "trpo_iters_per_sec": round(K / elapsed, 4),
        "rollout_env_steps_per_sec": round(n_local * world * K / (phases["rollout"] * 1e-3), 1),
        "phase_ms_per_iter": {k: round(v / K, 3) for k, v in phases.items()},
        "kernels": {k: {kk: (round(vv, 5) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in kinfo.items()},
        "roofline": roofline,
        "roofline_gae": gae,
        "roofline_policy_gemm": pg_roof,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(cpu_E, cpu_T, args.env, hid)
        line["cpu_baseline"]["serial_c1"] = cpu_serial_c1()
    json_out.write(json.dumps(line) + "\n")
    json_out.flush()
    return runner


def _release(runner):
    """Drop the captured rollout graph, device buffers and the CU-masked streams before
    interpreter teardown: a stream left to the HIP runtime's own teardown is destroyed
    after an attached rocprofv3 has finalised, which crashed the process at exit
    (tools/teardown_probe.py)."""
    if runner is not None:
        runner.col.graph = None
    del runner
    gc.collect()
    if torch.cuda.is_available():
        from modular_rl_amd import streams
        streams.destroy_all()
        torch.cuda.empty_cache()
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    _release(main())
