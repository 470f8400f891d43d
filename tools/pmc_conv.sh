#!/bin/bash
# SQ counter passes over the conv micro-bench (one rocprofv3 --pmc pass per counter group; the
# guide's slot limits: <= 8 SQ counters per pass).  Usage: tools/pmc_conv.sh OUTDIR "variants" "shapes"
set -e
OUT=$(realpath -m "$1"); V=${2:-5,6}; S=${3:-0}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
P3="SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_CYCLES SQ_INSTS_BRANCH"
P4="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pass$i" -o run -- \
    python3 "$ROOT/tools/conv_bench.py" --variants "$V" --shapes "$S" --reps 2 --rounds 1 --gn > "$OUT/pass$i.log" 2>&1
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"/pass*/run_counter_collection.csv --kernels conv_halo > "$OUT/summary.json"
