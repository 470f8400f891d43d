#!/bin/bash
# Interleaved A/B of conv micro-bench timings across library builds (tools/build_variant.py):
#   tools/ab_conv.sh OUTDIR ROUNDS SHAPES lib1 lib2 ...   (each lib path, or "default")
# Every (round, lib) runs tools/conv_bench.py --gn in its own process under a 120 s limit.
OUT=$1; ROUNDS=$2; SHAPES=$3; shift 3
mkdir -p "$OUT"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    tag=$(basename "$(dirname "$lib")")
    [ "$lib" = default ] && tag=default
    if [ "$lib" = default ]; then
      timeout -k 10 120 python3 "$ROOT/tools/conv_bench.py" --gn --rounds 1 --reps 10 --shapes "$SHAPES" > "$OUT/r${r}_$tag.jsonl" 2> "$OUT/r${r}_$tag.err" || exit $?
    else
      SNRSE_LIB=$lib timeout -k 10 120 python3 "$ROOT/tools/conv_bench.py" --gn --rounds 1 --reps 10 --shapes "$SHAPES" > "$OUT/r${r}_$tag.jsonl" 2> "$OUT/r${r}_$tag.err" || exit $?
    fi
    echo "round $r $tag done" 
  done
done
