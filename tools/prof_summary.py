#!/usr/bin/env python3
"""Condense a rocprofv3 --stats kernel_stats.csv into markdown tables (top kernels, kernel families)."""
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
    # kernel families (all template instances of one kernel): the figure bench.py's roofline probe
    # reports as avg_launch_us for the dominant family
    fam = {}
    for r in rows:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0]
        c, t = fam.get(name, (0, 0.0))
        fam[name] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    lines += ["", "| kernel family (all instances) | calls | total ms | ms/step | avg us | % |", "|---|---|---|---|---|---|"]
    for name, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:8]:
        lines.append(f"| `{name}` | {c} | {t / 1e6:.1f} | {t / 1e6 / steps:.1f} | {t / c / 1e3:.1f} | {100 * t / tot:.1f} |")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, steps=int(sys.argv[3]) if len(sys.argv) > 3 else 1)
