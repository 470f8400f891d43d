#!/usr/bin/env python3
"""Per-shape attribution of a rocprofv3 --kernel-trace CSV: dispatches grouped by (kernel instance, grid
size), with count, mean / min / max duration and their share of the traced kernel time.  The halo GEMMs
launch one workgroup per 256-px x 128-cout tile, so the grid size names the level (C2, B = 32: 16384 =
level 0 at 128 couts, 4096 = level 1, ...).
Usage: python tools/dispatch_shapes.py run_kernel_trace.csv [SUBSTR] > out.jsonl"""
import collections
import csv
import json
import sys


def main(path, sub=""):
    groups = collections.OrderedDict()
    total = 0
    for r in csv.DictReader(open(path)):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        total += d
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if sub and sub not in name:
            continue
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        k = (name, grid // max(wg, 1))
        groups.setdefault(k, []).append(d)
    rows = []
    for (name, nwg), ds in groups.items():
        rows.append({"kernel": name, "workgroups": nwg, "count": len(ds), "mean_us": sum(ds) / len(ds) / 1e3,
                     "min_us": min(ds) / 1e3, "max_us": max(ds) / 1e3, "total_ms": sum(ds) / 1e6,
                     "share": sum(ds) / total if total else 0.0})
    for r in sorted(rows, key=lambda r: -r["total_ms"]):
        print(json.dumps(r))


if __name__ == "__main__":
    main(*sys.argv[1:])
