#!/usr/bin/env python3
"""Condense a rocprofv3 --kernel-trace database (rocpd sqlite, the default output format) into the
markdown kernel-stats table tools/prof_summary.py makes from the CSV format, plus a per-grid
breakdown of one kernel (the launches of different layer shapes have different durations).
Usage: tools/rocpd_summary.py RESULTS.db OUT.md [STEPS] [KERNEL_SUBSTRING]"""
import collections
import sqlite3
import sys


def main(db, out, steps=1, focus=None, top=25):
    c = sqlite3.connect(db)
    by = collections.defaultdict(lambda: [0, 0.0])
    grids = collections.defaultdict(lambda: [0, 0.0])
    for name, gx, wx, dur in c.execute("select name, grid_x, workgroup_x, duration from kernels"):
        short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
        by[short][0] += 1
        by[short][1] += dur
        if focus and focus in name:
            grids[gx // max(wx, 1)][0] += 1
            grids[gx // max(wx, 1)][1] += dur
    tot = sum(v[1] for v in by.values())
    lines = [f"source: `{db}` (rocprofv3 --kernel-trace --stats; steps profiled: {steps})", "",
             "| kernel | calls | total ms | ms/step | avg us | % |", "|---|---|---|---|---|---|"]
    for k, (n, t) in sorted(by.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"| `{k}` | {n} | {t / 1e6:.1f} | {t / 1e6 / steps:.1f} | {t / n / 1e3:.1f} | {100 * t / tot:.1f} |")
    lines.append(f"| **total** | | {tot / 1e6:.1f} | {tot / 1e6 / steps:.1f} | | 100 |")
    if focus:
        ft = sum(v[1] for v in grids.values())
        fn = sum(v[0] for v in grids.values())
        lines += ["", f"`{focus}` by grid (workgroups): {fn} launches, avg {ft / max(fn, 1) / 1e3:.1f} us", "",
                  "| workgroups | calls | avg us | % of kernel |", "|---|---|---|---|"]
        for g, (n, t) in sorted(grids.items(), key=lambda kv: -kv[1][1]):
            lines.append(f"| {g} | {n} | {t / n / 1e3:.1f} | {100 * t / ft:.1f} |")
    txt = "\n".join(lines) + "\n"
    open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    a = sys.argv
    main(a[1], a[2], int(a[3]) if len(a) > 3 else 1, a[4] if len(a) > 4 else None)
