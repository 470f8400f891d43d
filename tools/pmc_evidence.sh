#!/bin/bash
# One GPU call: HBM traffic per launch (FETCH_SIZE / WRITE_SIZE passes, N=2 bench) of the dominant conv kernel
# of the bf16 (conv_halo5_kernel) and fp32x3 (conv_x3h_kernel) C2 lines, and the fp32x3 probe-vs-rocprof
# reconciliation (kernel trace + the probe's per-call dump).  Usage: tools/pmc_evidence.sh TAG
set -e
TAG=$1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for DT in bf16 fp32x3; do
  K=conv_halo5_kernel; [ $DT = fp32x3 ] && K=conv_x3h_kernel
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/${DT}_$C" -o run -- \
      python3 "$ROOT/bench.py" --dtype $DT --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity > "$OUT/${DT}_$C.log" 2>&1
  done
  python3 "$ROOT/tools/pmc_traffic.py" "$OUT/${DT}_FETCH_SIZE/run_counter_collection.csv" \
    "$OUT/${DT}_WRITE_SIZE/run_counter_collection.csv" $K "$OUT/${DT}_pmc_traffic.json"
  rm -rf "$OUT/${DT}_FETCH_SIZE" "$OUT/${DT}_WRITE_SIZE"
done
SNRSE_PROBE_DUMP=$OUT/x3_probe_dump.json timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/x3trace" -o run -- \
  python3 "$ROOT/bench.py" --dtype fp32x3 --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-parity > "$OUT/x3_traced.json" 2> "$OUT/x3_traced.err"
python3 "$ROOT/tools/probe_reconcile.py" "$OUT/x3trace/run_kernel_trace.csv" "$OUT/x3_traced.json" "$OUT/x3_probe_vs_rocprof.json" "$OUT/x3_probe_dump.json"
rm -rf "$OUT/x3trace"
echo done > $OUT/DONE
