#!/bin/bash
# C5 ("long-form 30 s utterances, N=200, fp32: HBM-bound stress; rocprof roofline report", BASELINE configs[4]):
#   1. rocprofv3 --kernel-trace --stats of bench.py --config c5 --N 2 (with the in-bench roofline probe, so the
#      probe's per-launch figure and rocprof's can be reconciled on the same launches)
#   2. kernel-trace + FETCH_SIZE + WRITE_SIZE passes of one short identical command (--N 1, no probe), paired per
#      dispatch by tools/hbm_pairs.py -> measured HBM bytes and bandwidth per kernel and layer shape
# Usage: tools/c5_report.sh TAG      (outputs under gpurun_out/TAG)
set -e
TAG=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SNRSE_PROBE_DUMP=$OUT/probe_dump.json timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$ROOT/bench.py" --config c5 --N 2 --steps 1 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
python3 "$ROOT/tools/prof_summary.py" "$OUT/stats/run_kernel_stats.csv" "$OUT/kernel_stats.md" 3 > /dev/null
python3 "$ROOT/tools/probe_reconcile.py" "$OUT/stats/run_kernel_trace.csv" "$OUT/bench_traced.json" "$OUT/probe_vs_rocprof.json" \
  "$OUT/probe_dump.json"
rm -f "$OUT/stats/run_kernel_trace.csv"
CMD="python3 $ROOT/bench.py --config c5 --N 1 --steps 1 --warmup 0 --no-cpu-baseline --no-probe --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $CMD > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $CMD > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/hbm_pairs.py" "$OUT/trace/run_kernel_trace.csv" "$OUT/fetch/run_counter_collection.csv" \
  "$OUT/write/run_counter_collection.csv" "$OUT/hbm_pairs.json" conv_mfma gn_apply gn_act conv_splitk gn_stats attn \
  score_update conv_head > "$OUT/hbm_pairs.log"
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/fetch/run_counter_collection.csv" "$OUT/write/run_counter_collection.csv" \
  conv_mfma_kernel "$OUT/pmc_traffic.json" > /dev/null
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
echo done > "$OUT/DONE"
