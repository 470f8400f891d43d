#!/usr/bin/env python3
"""Instruction-class counts of one kernel in a device assembly file (hipcc --cuda-device-only -S).
Usage: tools/isa_stats.py file.s kernel_substring [--dump out.s]"""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
names = [m.group(1) for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", s, re.M) if pat in m.group(1) and not m.group(1).startswith(".")]
for name in names:
    a = s.index(name + ":")
    b = s.index(".Lfunc_end", a)
    body = s[a:b].split("\n")
    if "--dump" in sys.argv:
        open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(body))
    c = Counter()
    for l in body:
        l = l.strip()
        if not l or l.startswith((";", ".", "//")) or l.endswith(":"):
            continue
        op = l.split()[0]
        if op.startswith("v_mfma"): k = "mfma"
        elif op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq")): k = "trans"
        elif op.startswith(("v_writelane", "v_readlane")): k = "lane_spill"
        elif op.startswith("v_"): k = "valu"
        elif op.startswith("s_waitcnt"): k = "waitcnt"
        elif op.startswith("s_"): k = "salu"
        elif op.startswith("ds_"): k = "ds"
        elif op.startswith(("buffer_", "global_")): k = "vmem"
        else: k = op
        c[k] += 1
    print(name[:60], dict(sorted(c.items())))
