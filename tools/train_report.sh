#!/bin/bash
# --config train evidence: the bench line (with the CPU oracle leg) and a rocprofv3 --kernel-trace --stats
# summary of the training step's kernels (forward, dgrad, wgrad, GroupNorm backward, Adam).  Usage:
# tools/train_report.sh TAG    (outputs under gpurun_out/TAG)
set -e
TAG=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --config train --steps 3 --warmup 1 > "$OUT/train_line.json" 2> "$OUT/train_line.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$ROOT/bench.py" --config train --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/train_traced.json" 2> "$OUT/train_traced.err"
python3 "$ROOT/tools/prof_summary.py" "$OUT/stats/run_kernel_stats.csv" "$OUT/kernel_stats.md" 3 > /dev/null
rm -f "$OUT/stats/run_kernel_trace.csv"
echo done > "$OUT/DONE"
