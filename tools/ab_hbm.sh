#!/bin/bash
# Interleaved A/B of tools/hbm_bench.py across library builds: tools/ab_hbm.sh OUTDIR ROUNDS ONLY lib1 lib2 ...
# ("default" = the in-tree library); each run in its own process under a 150 s limit.
OUT=$1; ROUNDS=$2; ONLY=$3; shift 3
mkdir -p "$OUT"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    tag=$(basename "$(dirname "$lib")"); [ "$lib" = default ] && tag=default
    if [ "$lib" = default ]; then
      timeout -k 10 150 python3 "$ROOT/tools/hbm_bench.py" --only "$ONLY" --reps 10 > "$OUT/r${r}_$tag.jsonl" 2> "$OUT/r${r}_$tag.err" || exit $?
    else
      SNRSE_LIB=$lib timeout -k 10 150 python3 "$ROOT/tools/hbm_bench.py" --only "$ONLY" --reps 10 > "$OUT/r${r}_$tag.jsonl" 2> "$OUT/r${r}_$tag.err" || exit $?
    fi
  done
done
