#!/usr/bin/env python3
"""Pair rocprofv3 kernel-trace durations with FETCH_SIZE / WRITE_SIZE counters per dispatch for the
HBM-bound kernels (three runs of the same deterministic command: --kernel-trace, --pmc FETCH_SIZE,
--pmc WRITE_SIZE; dispatches of one kernel are matched by their order).  Groups by kernel and grid size
(= one layer shape) and reports the measured HBM bytes per launch, the mean duration and the achieved
bandwidth against 8 TB/s.  FETCH_SIZE is doubled (the gfx950 half-count correction of
MI355X_MICROARCH.md; calibrated for 16-B-per-lane streaming reads).

Usage: tools/hbm_pairs.py TRACE.csv FETCH.csv WRITE.csv OUT.json substr [substr ...]"""
import collections
import csv
import json
import sys

PEAK = 8.0e12


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()


def trace_rows(path, subs):
    out = collections.defaultdict(list)
    rd = csv.DictReader(open(path))
    keys = rd.fieldnames or []
    ks = next(k for k in keys if "Start" in k and "Timestamp" in k)
    ke = next(k for k in keys if "End" in k and "Timestamp" in k)
    kg = next((k for k in keys if k in ("Grid_Size_X", "Grid_Size", "Grid_X")), None)
    for r in rd:
        n = short(r["Kernel_Name"])
        if any(s in n for s in subs):
            grid = int(r[kg]) if kg and r[kg] else 0
            out[n].append((int(r[ke]) - int(r[ks]), grid))
    return out


def pmc_rows(path, counter, subs):
    vals = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = short(r["Kernel_Name"])
        if any(s in n for s in subs):
            d = vals[n]
            k = int(r["Dispatch_Id"])
            d[k] = d.get(k, 0.0) + float(r["Counter_Value"])
    return {n: [d[k] for k in sorted(d)] for n, d in vals.items()}


def main(trace, fetch, write, out, *subs):
    tr = trace_rows(trace, subs)
    fe = pmc_rows(fetch, "FETCH_SIZE", subs)
    wr = pmc_rows(write, "WRITE_SIZE", subs)
    res = []
    for n, rows in sorted(tr.items()):
        f, w = fe.get(n, []), wr.get(n, [])
        m = min(len(rows), len(f), len(w))
        groups = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
        for i in range(m):
            dur, grid = rows[i]
            g = groups[grid]
            g[0] += 1
            g[1] += dur
            g[2] += 2.0 * 1024.0 * f[i]
            g[3] += 1024.0 * w[i]
        for grid, (cnt, dur, fb, wb) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
            byt = (fb + wb) / cnt
            us = dur / cnt / 1e3
            res.append({"kernel": n, "grid": grid, "launches": cnt, "avg_us": us, "fetch_bytes": fb / cnt,
                        "write_bytes": wb / cnt, "hbm_bytes": byt, "TBps": byt / (us * 1e-6) / 1e12,
                        "frac_of_8TBps": byt / (us * 1e-6) / PEAK})
    with open(out, "w") as fh:
        json.dump({"note": "per (kernel, grid) group: measured HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) / mean "
                           "kernel-trace duration; three runs of the same command matched by dispatch order",
                   "groups": res}, fh, indent=1)
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main(*sys.argv[1:])
