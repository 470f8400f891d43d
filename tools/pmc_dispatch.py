#!/usr/bin/env python3
"""Per-dispatch counter values from a rocprofv3 --pmc counter_collection CSV, in dispatch order, for the
kernels whose name contains a substring.  Usage: python tools/pmc_dispatch.py CSV COUNTER SUBSTR [scale]"""
import collections
import csv
import json
import sys


def main(path, counter, sub, scale=1.0):
    vals = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or sub not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        d = vals.setdefault(k, [name, 0.0])
        d[1] += float(r["Counter_Value"])
    for k in sorted(vals):
        print(json.dumps({"dispatch": k, "kernel": vals[k][0], counter: vals[k][1],
                          "bytes": vals[k][1] * 1024.0 * float(scale)}))


if __name__ == "__main__":
    main(*sys.argv[1:])
