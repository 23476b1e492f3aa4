"""Summarise one rocprofv3 --pmc pass of SQ counters per kernel (means per launch) and
the wave-time split the DESIGN notes quote.

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
            -d OUT -o run --output-format csv -- python3 tools/fvp_probe.py
  python tools/sq_split.py OUT [kernel-substring ...]

WAVE / WAIT / ACTIVE count quad-cycles summed over waves; MFMA_BUSY counts cycles
summed over the SIMDs (1024 on MI355X): wait = s_waitcnt-parked, issue-stall =
waiting to issue (MFMA pipe busy or a dependency), active = issuing."""
import collections
import csv
import glob
import os
import sys

SIMDS = 1024


def main():
    d = sys.argv[1]
    keep = sys.argv[2:]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if keep and not any(k in name for k in keep):
                    continue
                acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name].add(r["Dispatch_Id"])
    for name, c in acc.items():
        n = len(disp[name])
        m = {k: v / n for k, v in c.items()}
        print(f"{name[:90]}  ({n} launches)")
        for k in sorted(m):
            print(f"  {k:28s} {m[k]:.4g}")
        w = m.get("SQ_WAVE_CYCLES", 0.0)
        if w > 0:
            wait = m.get("SQ_WAIT_ANY", 0.0) / w
            stall = m.get("SQ_WAIT_INST_ANY", 0.0) / w
            act = m.get("SQ_ACTIVE_INST_ANY", 0.0) / w
            print(f"  split of wave time: wait {wait:.2f}  issue-stall {stall:.2f}  active {act:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            print(f"  MFMA busy cycles per SIMD {m['SQ_VALU_MFMA_BUSY_CYCLES'] / SIMDS:.4g}")
        print()


if __name__ == "__main__":
    main()
