"""Per-step timeline of the layered rollout (Humanoid) from a rocprofv3 --kernel-trace CSV.

Takes the stream that runs the step kernel (default hm_act_kernel) and splits it into
steps at each step-kernel launch.  For every kernel position inside a step it reports
the mean duration and the mean gap before it (end of the previous kernel on that
stream to its start), plus the step-to-step period: how much of a step is kernel time
and how much is launch gap.

    python tools/step_timeline.py run_kernel_trace.csv [step_kernel_substring]
"""
import csv
import sys
from collections import defaultdict


def main(path, key="hm_act_kernel"):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"].split("(")[0].replace("void ", "")[:60], r["Stream_Id"]))
    sids = {sid for s, e, n, sid in rows if key in n}
    if not sids:
        print("no", key, "launches")
        return
    for sid in sorted(sids):
        ks = sorted((s, e, n) for s, e, n, q in rows if q == sid)
        steps, cur = [], []
        for k in ks:
            cur.append(k)
            if key in k[2]:
                steps.append(cur)
                cur = []
        # the first step of each rollout carries the reset; keep steps of the modal length
        lens = defaultdict(int)
        for st in steps:
            lens[len(st)] += 1
        L = max(lens, key=lens.get)
        use = [st for st in steps if len(st) == L]
        dur = [0.0] * L
        gap = [0.0] * L
        prev_end = None
        per = []
        for st in use:
            for i, (s, e, n) in enumerate(st):
                dur[i] += (e - s) / 1e3
                if i > 0:
                    gap[i] += (s - st[i - 1][1]) / 1e3
            per.append((st[-1][1] - st[0][0]) / 1e3)
        n = len(use)
        print(f"stream {sid}: {n} steps of {L} launches (of {len(steps)})")
        for i in range(L):
            print(f"  {use[0][i][2]:60s} dur {dur[i] / n:8.1f} us  gap before {gap[i] / n:6.1f} us")
        # period: start of step's first kernel to the next step's first kernel
        starts = [st[0][0] for st in use]
        p = [(b - a) / 1e3 for a, b in zip(starts, starts[1:]) if 0 < (b - a) / 1e3 < 5000]
        print(f"  first-to-last kernel span {sum(per) / n:.1f} us; step period {sum(p) / max(len(p), 1):.1f} us")
        print(f"  kernel time {sum(dur) / n:.1f} us, gaps {sum(gap) / n:.1f} us per step")


if __name__ == "__main__":
    main(*sys.argv[1:])
