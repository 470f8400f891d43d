#!/usr/bin/env python3
"""Reconcile bench.py's in-run roofline probe (HIP events around each probed conv call) with rocprofv3's
kernel trace of the same run.  The probe pass is the last enhancement of the process, so its conv calls
are the last `launches_per_pass` dispatches of the probed kernel in the trace.  A probed call can launch
more than one kernel (a split-K GEMM + conv_splitk_finalize), and its event bracket also holds the gap
between them, so three rocprof figures are reported for those calls: the GEMM kernel alone, GEMM +
its finalize, and first-start -> last-end of the call's kernels.

With the probe's per-call dump (bench.py under SNRSE_PROBE_DUMP=PATH) every probed conv2d call is matched to
its kernels in the trace (the conv launches of the probe pass, in order) and the per-call differences are
summarised by call duration.

Usage: tools/probe_reconcile.py KERNEL_TRACE.csv BENCH_LINE.json OUT.json [PROBE_DUMP.json]"""
import csv
import json
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0].strip()


CONV = ("conv_mfma_kernel", "conv_glds_kernel", "conv_halo5_kernel", "conv_head_kernel", "input_conv_kernel",
        "conv_x3_kernel", "conv_x3h_kernel")


def per_call(rows, dump):
    """Match the dumped probe calls (all conv2d calls of the pass, in order) with the trace's conv kernels."""
    calls = []  # (start, end) per conv call: a GEMM kernel and the split-K finalize kernels that follow it
    i = 0
    while i < len(rows):
        if rows[i][2] in CONV:
            s, e = rows[i][0], rows[i][1]
            j = i + 1
            while j < len(rows) and rows[j][2] == "conv_splitk_finalize":
                e = rows[j][1]
                j += 1
            calls.append((s, e))
            i = j
        else:
            i += 1
    n = len(dump["ms"])
    calls = calls[-n:]
    diffs = []
    for (s, e), ms, fl in zip(calls, dump["ms"], dump["flops"]):
        diffs.append((ms * 1e3, (e - s) / 1e3, fl is not None))
    buckets = {}
    for ev, rp, big in diffs:
        k = "<50us" if rp < 50 else ("50-500us" if rp < 500 else ">=500us")
        b = buckets.setdefault(k, [0, 0.0, 0.0])
        b[0] += 1
        b[1] += ev
        b[2] += rp
    out = {k: {"calls": v[0], "probe_avg_us": v[1] / v[0], "rocprof_avg_us": v[2] / v[0],
               "excess_avg_us": (v[1] - v[2]) / v[0]} for k, v in buckets.items()}
    big = [(ev, rp) for ev, rp, b in diffs if b]
    out["probed_big_calls"] = {"calls": len(big), "probe_avg_us": sum(e for e, _ in big) / len(big),
                               "rocprof_avg_us": sum(r for _, r in big) / len(big),
                               "note": "the calls bench.py's roofline averages (flops recorded), matched one to one"}
    return out


def main(trace, bench, out, dump=None):
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    roof = line["roofline"]
    kern, n = roof["kernel"], int(roof["launches_per_pass"])
    rd = csv.DictReader(open(trace))
    ks = next(k for k in rd.fieldnames if "Start" in k and "Timestamp" in k)
    ke = next(k for k in rd.fieldnames if "End" in k and "Timestamp" in k)
    rows = sorted(((int(r[ks]), int(r[ke]), short(r["Kernel_Name"])) for r in rd), key=lambda r: r[0])
    idx = [i for i, r in enumerate(rows) if r[2] == kern]
    if len(idx) < n:
        raise SystemExit(f"{kern}: {len(idx)} dispatches in the trace, probe saw {n}")
    idx = idx[-n:]
    alone, with_fin, span = [], [], []
    for i in idx:
        s, e, _ = rows[i]
        alone.append(e - s)
        j = i + 1
        fe = e
        fin = 0
        while j < len(rows) and rows[j][2] == "conv_splitk_finalize":
            fin += rows[j][1] - rows[j][0]
            fe = rows[j][1]
            j += 1
        with_fin.append(e - s + fin)
        span.append(fe - s)
    us = lambda v: sum(v) / len(v) / 1e3  # noqa: E731
    res = {"kernel": kern, "probe_calls": n, "probe_avg_us": roof["avg_launch_us"],
           "rocprof_kernel_alone_avg_us": us(alone), "rocprof_kernel_plus_finalize_avg_us": us(with_fin),
           "rocprof_call_span_avg_us": us(span),
           "calls_with_splitk_finalize": sum(1 for a, b in zip(alone, with_fin) if b > a),
           "note": "rocprof_* here average the LAST probe_calls dispatches of the kernel family, which is not the "
                   "probed set when small calls of the same kernel (1x1, Cout <= 16 heads) interleave; "
                   "per_call_by_duration matches every call one to one"}
    if dump:
        res["per_call_by_duration"] = per_call(rows, json.load(open(dump)))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
