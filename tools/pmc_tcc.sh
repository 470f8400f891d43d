#!/bin/bash
# L2 (TCC) hit / miss and HBM-side bytes of the conv micro-bench, one rocprofv3 --pmc pass per counter group
# (TCC_HIT + TCC_MISS; FETCH_SIZE; WRITE_SIZE: FETCH_SIZE takes 3 of the 4 TCC slots, so each its own pass).
# Usage: tools/pmc_tcc.sh OUTDIR "variants" "shapes" [--gn]
set -e
OUT=$(realpath -m "$1"); V=${2:-5,10}; S=${3:-1}; GN=${4:---gn}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pass$i" -o run -- \
    python3 "$ROOT/tools/conv_bench.py" --variants "$V" --shapes "$S" --reps 2 --rounds 1 $GN > "$OUT/pass$i.log" 2>&1
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT"/pass*/run_counter_collection.csv --kernels conv_halo > "$OUT/summary.json"
rm -rf "$OUT"/pass*/run_counter_collection.csv
