"""Issue floor of the persistent rollout's step from one rocprofv3 SQ pass.

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY \
              SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d OUT -o run -- python3 bench.py ...
    python tools/rollout_issue.py OUT KEY HORIZON [--out profiles/rollout_issue_r03.json]

The step is a latency chain of one wave per SIMD, so the time it cannot beat without
removing instructions is the wave's own issue time: SQ_ACTIVE_INST_ANY (quad-cycles,
summed over waves; MI355X_MICROARCH.md § rocprofv3 PMC slots) x 4 / (waves x steps)
cycles per step.  KEY names the bench line (e.g. Hopper-v2/fp32); entries merge into
the JSON file bench.py reads for its rollout roofline."""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("key")
    ap.add_argument("horizon", type=int)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    acc = collections.defaultdict(float)
    disp = set()
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "rollout_persistent_kernel" not in r["Kernel_Name"]:
                    continue
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
    if not disp:
        raise SystemExit("no rollout_persistent_kernel dispatches")
    n = len(disp)
    m = {k: v / n for k, v in acc.items()}  # per launch
    waves = m["SQ_WAVES"]
    per = lambda c: m[c] / (waves * a.horizon)  # noqa: E731  per wave per step
    e = {"launches": n, "waves_per_launch": waves, "horizon": a.horizon,
         "issue_cycles_per_step": 4 * per("SQ_ACTIVE_INST_ANY"),
         "wave_cycles_per_step": 4 * per("SQ_WAVE_CYCLES"),
         "issue_stall_cycles_per_step": 4 * per("SQ_WAIT_INST_ANY"),
         "waitcnt_cycles_per_step": 4 * per("SQ_WAIT_ANY"),
         "valu_insts_per_step": per("SQ_INSTS_VALU"), "salu_insts_per_step": per("SQ_INSTS_SALU"),
         "lds_insts_per_step": per("SQ_INSTS_LDS"),
         "note": "per wave per step of rollout_persistent_kernel; SQ_* quad-cycles x4 = cycles; "
                 "counters summed over all waves of a launch, divided by SQ_WAVES x horizon"}
    out = {}
    if a.out and os.path.exists(a.out):
        with open(a.out) as fh:
            out = json.load(fh)
    out[a.key] = e
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    print(json.dumps({a.key: e}, indent=1))


if __name__ == "__main__":
    main()
