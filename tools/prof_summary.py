#!/usr/bin/env python3
"""Condense a rocprofv3 --stats kernel_stats.csv into a markdown table (top kernels)."""
import csv
import sys


def main(path, out=None, top=25, steps=1):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"source: `{path}` (steps profiled: {steps})", "",
             "| kernel | calls | total ms | ms/step | avg us | % |", "|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        lines.append(f"| `{name}` | {r['Calls']} | {t / 1e6:.1f} | {t / 1e6 / steps:.1f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    lines.append(f"| **total** | | {tot / 1e6:.1f} | {tot / 1e6 / steps:.1f} | | 100 |")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, steps=int(sys.argv[3]) if len(sys.argv) > 3 else 1)
