#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 PMC counters per dispatch (counter_collection.csv files).

  python tools/pmc_summary.py OUT/pass*/run_counter_collection.csv [--kernels conv_halo5,conv_halo6]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--kernels", default="")
    a = ap.parse_args()
    pref = [k for k in a.kernels.split(",") if k]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> counter -> sum
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in a.files:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = name.split("(")[0].replace("void ", "").strip()
            if pref and not any(name.split("<")[0].split("::")[-1].startswith(p) for p in pref):
                continue
            c = r["Counter_Name"]
            acc[name][c] += float(r["Counter_Value"])
            disp[name][c].add(r["Dispatch_Id"])
    out = {}
    for k, d in acc.items():
        out[k] = {c: v / max(1, len(disp[k][c])) for c, v in sorted(d.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
