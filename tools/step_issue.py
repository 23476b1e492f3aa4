"""Issue floor of the layered (Humanoid) rollout step from one rocprofv3 SQ pass over
tools/humanoid_collect.py (every dispatch of that run belongs to the rollout):

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY \
              SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d OUT -o run -- \
              python3 tools/humanoid_collect.py E T [dtype]
    python tools/step_issue.py OUT KEY [--out profiles/rollout_issue_r04.json]

A step is a chain of dependent launches: the filter merge + normalised obs
(lrollout_obs_kernel), the bf16 cast of the obs rows, the hidden-layer GEMMs
(gemm_bf16_small_kernel) and the env step with the fused head (hm_act_kernel, one wave
per env) and the block partials (lrollout_partials_kernel).  No launch of the chain can
finish before its waves have issued their instructions, so the step's floor is the sum
over its launches of the issue time of one wave (SQ_ACTIVE_INST_ANY quad-cycles x 4 /
SQ_WAVES: the waves run side by side, one per SIMD for the env step); the launch gaps and
every wait are what the achieved step time adds.  Steps = hm_act_kernel dispatches."""
import argparse
import collections
import csv
import glob
import json
import os

STEP_KERNELS = ("lrollout_obs_kernel", "cast_rows_bf16_kernel", "gemm_bf16_small_kernel", "gemm_f32_kernel",
                "hm_act_kernel", "lrollout_partials_kernel")


def short(name):
    # "void mrl::gemm_bf16_small_kernel<true>(...)" -> "gemm_bf16_small_kernel"
    return name.split("(")[0].split("<")[0].replace("void ", "").strip().split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("key")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # dispatch -> counter -> value
    kname = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if k not in STEP_KERNELS:
                    continue
                d = (f, r["Dispatch_Id"])
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
                kname[d] = k
    steps = sum(1 for d in per if kname[d] == "hm_act_kernel")
    if not steps:
        raise SystemExit("no hm_act_kernel dispatches")
    kern = collections.defaultdict(lambda: collections.defaultdict(float))
    for d, c in per.items():
        w = max(c["SQ_WAVES"], 1.0)
        e = kern[kname[d]]
        e["dispatches"] += 1
        e["issue_cycles_per_wave"] += 4 * c["SQ_ACTIVE_INST_ANY"] / w
        e["wave_cycles_per_wave"] += 4 * c["SQ_WAVE_CYCLES"] / w
        e["waitcnt_cycles_per_wave"] += 4 * c["SQ_WAIT_ANY"] / w
        e["valu_insts_per_wave"] += c["SQ_INSTS_VALU"] / w
        e["salu_insts_per_wave"] += c["SQ_INSTS_SALU"] / w
        e["waves"] += w
    out_k = {}
    for k, e in kern.items():
        n = e["dispatches"]
        out_k[k] = {"per_step": n / steps, "waves_per_dispatch": e["waves"] / n,
                    **{x: e[x] / n for x in ("issue_cycles_per_wave", "wave_cycles_per_wave", "waitcnt_cycles_per_wave",
                                             "valu_insts_per_wave", "salu_insts_per_wave")}}
    floor = sum(v["per_step"] * v["issue_cycles_per_wave"] for v in out_k.values())
    e = {"steps": steps, "issue_cycles_per_step": floor,
         "valu_insts_per_step": sum(v["per_step"] * v["valu_insts_per_wave"] for v in out_k.values()),
         "kernels": out_k,
         "note": "layered rollout step = chain of launches; floor = sum over the step's launches of one wave's "
                 "issue cycles (SQ_ACTIVE_INST_ANY x4 / SQ_WAVES), launches per step = dispatches / hm_act dispatches"}
    out = {}
    if a.out and os.path.exists(a.out):
        with open(a.out) as fh:
            out = json.load(fh)
    out[a.key] = e
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(json.dumps(out, indent=1) + "\n")
    print(json.dumps({a.key: e}, indent=1))


if __name__ == "__main__":
    main()
