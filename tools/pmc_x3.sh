#!/bin/bash
# SQ counter passes over the split-bf16 halo GEMM (conv_x3h_kernel, fused GroupNorm+SiLU) on one x3_bench shape, one
# rocprofv3 --pmc pass per counter group (<= 8 SQ counters a pass).  Usage: tools/pmc_x3.sh OUTDIR [shape index]
set -e
OUT=$(realpath -m "$1"); S=${2:-0}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
P4="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pass$i" -o run -- \
    python3 "$ROOT/tools/x3_bench.py" --tiles 0 --exact 0 --gn 1 --reps 2 --shapes "$S" > "$OUT/pass$i.log" 2>&1
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"/pass*/run_counter_collection.csv --kernels conv_x3h > "$OUT/summary.json"
rm -f "$OUT"/pass*/run_counter_collection.csv
