#!/bin/bash
# interleaved A/B of tools/x3_bench.py across library builds: OUT ROUNDS lib...
OUT=$1; R=$2; shift 2; mkdir -p $OUT
for r in $(seq 1 $R); do for lib in "$@"; do
  tag=$(basename $(dirname $lib)); [ "$lib" = default ] && tag=default
  if [ "$lib" = default ]; then timeout -k 10 200 python3 tools/x3_bench.py --tiles 0 --exact 0 --gn 1 --spread 1 --reps 10 > $OUT/r${r}_$tag.jsonl 2> $OUT/r${r}_$tag.err || exit $?
  else SNRSE_LIB=$lib timeout -k 10 200 python3 tools/x3_bench.py --tiles 0 --exact 0 --gn 1 --spread 1 --reps 10 > $OUT/r${r}_$tag.jsonl 2> $OUT/r${r}_$tag.err || exit $?; fi
  echo "round $r $tag"; done; done
