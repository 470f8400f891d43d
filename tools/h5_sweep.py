#!/usr/bin/env python3
"""Sweep of the persistent / staggered v5 halo-GEMM launch options on the conv_bench shapes.
Usage (GPU box): python tools/h5_sweep.py [--gn] [--shapes 0,3] [--settings "0:0,1:0,1:3600"]
(setting = h5_persist:h5_stagger[:epi_nt]).  Outputs of every setting are compared with the first one."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from conv_bench import SHAPES, run  # noqa: E402
from snrse import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--shapes", default="0,1,2,3,4,5")
    ap.add_argument("--settings", default="0:0,1:0,1:2400,1:3600,1:4800")
    ap.add_argument("--gn", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    sets = [tuple(int(v) for v in s.split(":")) for s in a.settings.split(",")]
    for si in [int(x) for x in a.shapes.split(",")]:
        sh = SHAPES[si]
        row = {"shape": sh, "gn": a.gn}
        ref = None
        for rnd in range(2):
            for st in sets:
                pers, stg, nt = (list(st) + [0])[:3]
                ops.set_option("h5_persist", pers)
                ops.set_option("h5_stagger", stg)
                ops.set_option("epi_nt", nt)
                out, ms, fl = run(sh, 5, a.reps, dev, gn=a.gn)
                key = f"p{pers}_s{stg}_nt{nt}"
                row[key] = round(min(ms, row.get(key, ms)) * 1e3, 1)
                row[key + "_tf"] = round(fl / (row[key] * 1e-3) / 1e9, 1)
                if ref is None:
                    ref = out.float().clone()
                else:
                    row["maxdiff"] = max(row.get("maxdiff", 0.0), (out.float() - ref).abs().max().item())
        print(json.dumps(row), flush=True)
    ops.set_option("h5_persist", 0)
    ops.set_option("h5_stagger", 3600)
    ops.set_option("epi_nt", 0)


if __name__ == "__main__":
    main()
