#!/bin/bash
# One GPU call: bench.py line + rocprofv3 --kernel-trace --stats summary of one bench pass pair
# (1 warmup + 1 timed enhance pass, no probe / parity) for a dtype.
# Usage: tools/prof_x3.sh TAG [DTYPE=fp32x3] [extra bench args]
set -e
TAG=${1:-r03x3}; DT=${2:-fp32x3}; shift 2 || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --dtype $DT --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --dtype $DT --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-probe "$@" > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
python3 "$ROOT/tools/prof_summary.py" "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.md" 2 > /dev/null
rm -f "$OUT/trace/run_kernel_trace.csv"
echo done > $OUT/DONE
