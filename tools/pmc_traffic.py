"""HBM traffic per launch of the hot-path kernels from two rocprofv3 counter passes
(MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE need separate passes; gfx950's
FETCH_SIZE counts half the bytes of wide coalesced reads -> x2; both are in KB).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <fetch_dir> -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <write_dir> -o run -- python bench.py ...
    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/pmc_r01.json]
"""
import argparse
import csv
import glob
import json
import os

# role -> kernel-name substring (first match wins, most specific first)
ROLES = [
    ("pg_onepass", "mlp_fisher_hyb_kernel<1, 1>"),  # the one-launch policy gradient (round 6)
    ("pg_onepass", "mlp_fisher_hyb_kernel<2, 1>"),
    ("fvp_onepass", "mlp_fisher_hyb_kernel"),        # the one-pass Fisher product (round 5)
    ("fvp_jvp_rows_split", "mlp_fvp_split_kernel"),
    ("fvp_jvp_rows", "mlp_rows_kernel<100"),
    ("fvp_vjp", "mlp_vjp16_kernel<false, false"),  # the cached VJP (16-row kernel)
    ("fvp_vjp_r02", "mlp_vjp_kernel<true"),          # its round-2 32-row predecessor
    ("fvp_jvp_rows_bf16", "mlp_rows_bf16_kernel<100"),
    ("fvp_vjp_bf16", "mlp_vjp_bf16_kernel<true"),
    ("vjp_uncached", "mlp_vjp_kernel<false"),
    ("rows_surrgrad", "mlp_rows_kernel<2,"),
    ("rows_vfloss", "mlp_rows_kernel<3,"),
    ("rollout_persistent", "rollout_persistent_kernel"),
    ("rollout_step", "rollout_step_kernel"),
    ("gae_scan", "gae_full_kernel"),                  # the exact-fit GAE kernel (round 6)
    ("gae_scan", "gae_scan_kernel"),
    ("episode_stats", "episode_stats_kernel<"),
    ("gemm_nn", "gemm_f32_kernel<false, false, 128>"),
    ("gemm_nt", "gemm_f32_kernel<false, true, 128>"),
    ("gemm_tn", "gemm_f32_kernel<true, false, 128>"),
]


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def per_role(d, counter):
    acc = {}
    for r in _rows(d):
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "")
        for role, sub in ROLES:
            if sub in name:
                a = acc.setdefault(role, [0, 0.0])
                a[0] += 1
                a[1] += float(r["Counter_Value"])
                break
    return {k: (n, tot / n) for k, (n, tot) in acc.items()}


def gemm_dispatches(d, counter):
    vals = [float(r["Counter_Value"]) for r in _rows(d) if r.get("Counter_Name") == counter
            and "gemm" in r.get("Kernel_Name", "") and "cast_rows" not in r["Kernel_Name"]
            and "pack_w" not in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no GEMM dispatches with {counter} under {d}")
    return len(vals), sum(vals) / len(vals)


def gemm_entry(a):
    nf, f = gemm_dispatches(a.fetch_dir, "FETCH_SIZE")
    nw, w = gemm_dispatches(a.write_dir, "WRITE_SIZE")
    e = {"FETCH_SIZE_KB_mean": f, "WRITE_SIZE_KB_mean": w, "launches_FETCH_SIZE": nf, "launches_WRITE_SIZE": nw,
         "hbm_bytes_per_launch": int(round((2.0 * f + w) * 1024)),
         "note": "tools/gemm_pmc_probe.py on this one shape; FETCH_SIZE x2 (gfx950), KB->bytes, separate passes"}
    out = {}
    if a.out and os.path.exists(a.out):
        with open(a.out) as fh:
            out = json.load(fh)
    out.setdefault(a.key or "probe", {})[a.gemm] = e
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    print(json.dumps({a.gemm: e}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--horizon", type=int, default=1024,
                    help="steps per persistent rollout launch: its bytes / horizon = the per-step rollout_step figure")
    ap.add_argument("--gemm", default=None, help="a tools/gemm_pmc_probe.py label: average the probe's GEMM "
                                                 "dispatches (cast / pack setup kernels skipped) into --out[--key][label]")
    ap.add_argument("--key", default=None, help="bench line of the --gemm entry, e.g. Humanoid-v2/bf16/1024")
    a = ap.parse_args()
    if a.gemm:
        return gemm_entry(a)
    fe = per_role(a.fetch_dir, "FETCH_SIZE")
    wr = per_role(a.write_dir, "WRITE_SIZE")
    out = {}
    note = ("FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md HBM), KB->bytes x1024; "
            "separate --pmc passes")
    for role in sorted(set(fe) | set(wr)):
        f = fe.get(role)
        w = wr.get(role)
        e = {"note": note}
        if f:
            e["FETCH_SIZE_KB_mean"], e["launches_FETCH_SIZE"] = f[1], f[0]
        if w:
            e["WRITE_SIZE_KB_mean"], e["launches_WRITE_SIZE"] = w[1], w[0]
        if f and w:
            e["hbm_bytes_per_launch"] = int(round((2.0 * f[1] + w[1]) * 1024))
        out[role] = e
    if "rollout_persistent" in out and "hbm_bytes_per_launch" in out["rollout_persistent"]:
        out["rollout_step"] = {"note": f"rollout_persistent bytes / {a.horizon} steps (one launch runs the horizon)",
                               "hbm_bytes_per_launch": int(round(out["rollout_persistent"]["hbm_bytes_per_launch"]
                                                                 / a.horizon))}
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
