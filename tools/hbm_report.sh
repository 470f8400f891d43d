#!/bin/bash
# VERDICT r02 item 4 evidence: the same-box streaming calibration (tools/hbm_calib.hip) and, for the
# level-0 HBM-bound kernels (gn_resample down, input_conv, conv_head<2>), a timing run plus SQ counter
# and FETCH / WRITE passes of tools/hbm_bench.py.  Usage: tools/hbm_report.sh TAG   (outputs gpurun_out/TAG)
set -e
TAG=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$ROOT/tools/bin/hbm_calib" 10 > "$OUT/calib.jsonl" 2> "$OUT/calib.err"
CMD="python3 $ROOT/tools/hbm_bench.py --only down,input,head --levels 0 --reps 5"
timeout -k 10 200 $CMD > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU"
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/sq" -o run -- $CMD > "$OUT/sq.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $CMD > "$OUT/fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $CMD > "$OUT/write.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/grbm" -o run -- $CMD > "$OUT/grbm.log" 2>&1
python3 "$ROOT/tools/pmc_summary.py" "$OUT"/sq/run_counter_collection.csv "$OUT"/fetch/run_counter_collection.csv \
  "$OUT"/write/run_counter_collection.csv "$OUT"/grbm/run_counter_collection.csv \
  --kernels gn_resample_rows_kernel,input_conv_kernel,conv_head_kernel > "$OUT/pmc_summary.json"
rm -rf "$OUT/sq" "$OUT/fetch" "$OUT/write" "$OUT/grbm"
echo done > "$OUT/DONE"
