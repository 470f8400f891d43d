#!/bin/bash
# One profiling call on the GPU box (each step under its own time limit, stop at the first failure):
#   1. rocprofv3 --kernel-trace --stats of bench.py (TAG_bench_kernel_stats.*)
#   2. FETCH_SIZE / WRITE_SIZE passes over a short bench (N=2) -> per-launch HBM bytes of the halo GEMM
#   3. SQ counter passes of the halo GEMM on the level-0 Conv_0 shape (tools/pmc_conv.sh)
#   4. conv micro-bench over the NCSN++ shapes
# Usage: tools/profile_run.sh TAG [bench args...]
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BARGS="$@"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $BARGS > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
python3 "$ROOT/tools/prof_summary.py" "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.md" 3 > /dev/null
rm -f "$OUT/trace/run_kernel_trace.csv"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe $BARGS > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe $BARGS > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/fetch/run_counter_collection.csv" "$OUT/write/run_counter_collection.csv" \
  conv_halo5_kernel "$OUT/pmc_traffic.json"
bash "$ROOT/tools/pmc_conv.sh" "$OUT/sq" 5 0
timeout -k 10 300 python3 "$ROOT/tools/conv_bench.py" --variants 5 --rounds 2 --reps 10 --gn > "$OUT/conv_bench.jsonl" 2> "$OUT/conv_bench.err"
rm -rf "$OUT/fetch" "$OUT/write"  # large per-dispatch CSVs (the summary keeps what is used)
echo done > "$OUT/DONE"
