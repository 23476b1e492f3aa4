"""Per-role kernel durations from a rocprofv3 --kernel-trace CSV, with the Fisher-product
VJP told apart from the other launches of the same template: it is the mlp_vjp_kernel
dispatch that follows an mlp_rows_kernel<100 (FVP rows) dispatch on the same stream.
bench.py's live HIP-event averages (``kernels``, ``roofline``) are over exactly these.

    python tools/fvp_trace_stats.py <run_kernel_trace.csv>    (all launches, warmup included)
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    last_rows100 = {}
    for r in rows:
        n, s = r["Kernel_Name"], r["Stream_Id"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # ms
        if "mlp_rows_kernel<100" in n:
            dur["fvp_jvp_rows"].append(d)
            last_rows100[s] = True
        elif "mlp_vjp_kernel<true" in n:
            dur["fvp_vjp" if last_rows100.get(s) else "vjp_other"].append(d)
            last_rows100[s] = False
        elif "gae_scan_kernel" in n:
            dur["gae_scan"].append(d)
        elif "rollout_step_kernel" in n:
            dur["rollout_step"].append(d)
        elif "mlp_rows_kernel" in n:
            last_rows100[s] = False
    print(f"{'role':14s} {'launches':>8s} {'mean_ms':>10s} {'min_ms':>10s} {'max_ms':>10s}")
    for k in ("fvp_jvp_rows", "fvp_vjp", "vjp_other", "gae_scan", "rollout_step"):
        v = dur.get(k)
        if v:
            print(f"{k:14s} {len(v):8d} {sum(v) / len(v):10.4f} {min(v):10.4f} {max(v):10.4f}")


if __name__ == "__main__":
    main()
