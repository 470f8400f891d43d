#!/bin/bash
# Compact per-kernel resource usage (VGPR / SGPR / spills / occupancy) of one HIP source for gfx950.
# Usage: tools/kres.sh file.hip [name-filter] [extra hipcc flags...]
SRC=$1; FILT=${2:-.}; shift; shift
DIR=$(dirname "$SRC")
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -fno-slp-vectorize "$@" -I"$DIR" -c "$SRC" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
filt = sys.argv[1]
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"(VGPRs|AGPRs|TotalSGPRs|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "")] = int(m.group(2))
for k, v in rows.items():
    if re.search(filt, k):
        print(f"{k[:70]:70s} " + " ".join(f"{a}={b}" for a, b in v.items()))
' "$FILT"
