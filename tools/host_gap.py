"""GPU idle time at the iteration boundary, from a rocprofv3 --kernel-trace CSV.

For every launch of the rollout kernel (the start of an iteration's device work) it
reports the gap between the latest end of any kernel that started before it and the
rollout's start (negative = the rollout was issued while update kernels still ran, as
with the prelaunch of core.IterationRunner), plus the idle time of the whole device
(gaps in the union of all kernels' busy intervals) between consecutive rollout starts.

    python tools/host_gap.py run_kernel_trace.csv [rollout_kernel_substring]
"""
import csv
import sys


def main(path, key="rollout_persistent_kernel"):
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    starts = [s for s, _, n in ks if key in n]
    if len(starts) < 2:
        print(f"fewer than two '{key}' launches")
        return
    print(f"{'iter':>4} {'boundary_gap_us':>15} {'idle_us':>9} {'period_ms':>9}")
    gaps, idles = [], []
    for i, rs in enumerate(starts):
        before = [e for s, e, n in ks if s < rs]
        gap = (rs - max(before)) / 1e3 if before else float("nan")
        idle = float("nan")
        if i + 1 < len(starts):
            lo, hi = rs, starts[i + 1]
            busy_end, idle_ns = lo, 0
            for s, e, _ in ks:
                if e <= lo or s >= hi:
                    continue
                s, e = max(s, lo), min(e, hi)
                if s > busy_end:
                    idle_ns += s - busy_end
                busy_end = max(busy_end, e)
            idle_ns += max(0, hi - busy_end)
            idle = idle_ns / 1e3
            idles.append(idle)
        if i > 0:
            gaps.append(gap)
        per = (starts[i + 1] - rs) / 1e6 if i + 1 < len(starts) else float("nan")
        print(f"{i:4d} {gap:15.1f} {idle:9.1f} {per:9.3f}")
    if gaps:
        gs = sorted(gaps)
        print(f"boundary gap (iterations 1..): median {gs[len(gs) // 2]:.1f} us, max {gs[-1]:.1f} us")
    if idles:
        print(f"device idle per iteration: median {sorted(idles)[len(idles) // 2]:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
