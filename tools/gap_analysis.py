#!/usr/bin/env python3
"""GPU idle time between kernels from a rocprofv3 --kernel-trace CSV: sorts dispatches by start, merges
overlapping intervals, and reports busy vs idle time over the window and the gap histogram.
Usage: python tools/gap_analysis.py run_kernel_trace.csv [--skip-first-ms 0]"""
import csv
import json
import sys


def main(path, skip_ms=0.0):
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            iv.append((s, e, r.get("Kernel_Name", "")))
    iv.sort()
    t0 = iv[0][0] + int(skip_ms * 1e6)
    iv = [x for x in iv if x[0] >= t0]
    busy, gaps, cur_s, cur_e = 0, [], iv[0][0], iv[0][1]
    prev, where = iv[0][2], []
    for s, e, name in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            where.append((s - cur_e, (cur_e - iv[0][0]) / 1e6, prev[:60], name[:60]))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = name
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    gaps.sort()
    hist = {k: sum(1 for g in gaps if lo <= g < hi) for k, (lo, hi) in
            {"<1us": (0, 1000), "1-2us": (1000, 2000), "2-5us": (2000, 5000), "5-20us": (5000, 20000),
             ">=20us": (20000, 1 << 62)}.items()}
    print(json.dumps({"dispatches": len(iv), "span_ms": span / 1e6, "busy_ms": busy / 1e6,
                      "idle_ms": (span - busy) / 1e6, "idle_frac": (span - busy) / span,
                      "gaps": len(gaps), "median_gap_us": gaps[len(gaps) // 2] / 1e3 if gaps else 0,
                      "gap_hist": hist, "idle_in_gaps_ge_20us_ms": sum(g for g in gaps if g >= 20000) / 1e6}))
    from collections import Counter
    pairs = Counter((a, b) for g, _, a, b in where if g >= 5000)
    tot = Counter()
    for g, _, a, b in where:
        if g >= 5000:
            tot[(a, b)] += g / 1e3
    for (a, b), n in pairs.most_common(12):
        print(json.dumps({"after": a, "before": b, "count": n, "total_us": round(tot[(a, b)], 1)}))
    for g, t, a, b in sorted(where, reverse=True)[:8]:
        print(json.dumps({"gap_us": g / 1e3, "at_ms": round(t, 2), "after": a, "before": b}))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[3]) if len(sys.argv) > 3 else 0.0)
