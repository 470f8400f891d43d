#!/bin/bash
# PMC + kernel-trace pairs of the HBM-bound kernels over one short C2 bench (N=2): three runs of the same
# command, each under its own limit; tools/hbm_pairs.py matches them.  Usage: tools/hbm_pairs_run.sh TAG
set -e
TAG=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $ROOT/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity --no-parity-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $CMD > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $CMD > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/hbm_pairs.py" "$OUT/trace/run_kernel_trace.csv" "$OUT/fetch/run_counter_collection.csv" \
  "$OUT/write/run_counter_collection.csv" "$OUT/hbm_pairs.json" gn_resample input_conv conv_head gn_act > "$OUT/hbm_pairs.log"
head -1 "$OUT/trace/run_kernel_trace.csv" > "$OUT/trace_header.txt"
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
