"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite): per-dispatch listing of
the last N dispatches, or per-(kernel, grid) totals.

    python tools/prof_summary.py <run_results.db> [--last N] [--group] [--gaps US]

--gaps US: over the last N dispatches, the busy time, the idle time and every gap
longer than US microseconds between one dispatch's end and the next one's start.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--group", action="store_true")
    ap.add_argument("--gaps", type=float, default=None)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, accum_vgpr_count, "
                       "lds_size, scratch_size, start, end from kernels order by start").fetchall()
    short = lambda n: n.split("(")[0].replace("void ", "")[:60]
    if a.group:
        agg = {}
        for r in rows:
            k = (short(r[0]), r[2], r[3], r[4])
            c = agg.setdefault(k, [0, 0.0, r[6], r[7], r[8], r[9]])
            c[0] += 1
            c[1] += r[1]
        tot = sum(v[1] for v in agg.values())
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{v[1] / 1e6:9.3f} ms {100 * v[1] / tot:5.1f}% n={v[0]:4d} avg={v[1] / v[0] / 1e3:9.1f} us "
                  f"grid={k[1]}x{k[2]}x{k[3]} vgpr={v[2]}+{v[3]} lds={v[4]} scr={v[5]} {k[0]}")
    if a.gaps is not None:
        sel = rows[-a.last:] if a.last else rows
        busy = sum(r[1] for r in sel)
        span = sel[-1][11] - sel[0][10]
        print(f"span {span / 1e6:.3f} ms busy {busy / 1e6:.3f} ms idle {(span - busy) / 1e6:.3f} ms "
              f"over {len(sel)} dispatches")
        for prev, r in zip(sel, sel[1:]):
            g = (r[10] - prev[11]) / 1e3
            if g > a.gaps:
                print(f"gap {g:9.1f} us before {short(r[0])} (after {short(prev[0])})")
        return
    for r in rows[-a.last:] if a.last else []:
        print(f"{r[1] / 1e3:9.1f} us grid={r[2]}x{r[3]}x{r[4]} {short(r[0])}")


if __name__ == "__main__":
    main()
