"""Per-(kernel, stream) launch statistics from a rocprofv3 --kernel-trace CSV: with the
pipelined loop the VF fit's kernels run on a CU-masked stream beside the rollout, so
their durations are reported apart from the same kernels on the iteration stream.

    python tools/trace_by_stream.py run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def main(path):
    agg = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[(name, r["Stream_Id"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'total_ms':>9} {'share':>6} {'calls':>6} {'avg_us':>9} {'min_us':>8} stream kernel")
    for (name, sid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) / tot < 0.001:
            continue
        print(f"{sum(v) / 1e3:9.3f} {100 * sum(v) / tot:5.1f}% {len(v):6d} {sum(v) / len(v):9.1f} {min(v):8.1f} "
              f"{sid:>6} {name[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
