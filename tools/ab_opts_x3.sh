#!/bin/bash
OUT=gpurun_out/r03zZd_x3opts; mkdir -p $OUT
for r in 1 2; do
  for o in none splitk_target=512 splitk_target=128 x3_tile=4; do
    if [ $o = none ]; then timeout -k 10 200 python -u bench.py --dtype fp32x3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-probe > $OUT/r${r}_$o.log 2>&1 || exit $?
    else SNRSE_OPTS=$o timeout -k 10 200 python -u bench.py --dtype fp32x3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-probe > $OUT/r${r}_$o.log 2>&1 || exit $?; fi
    echo "round $r $o $(grep '^{' $OUT/r${r}_$o.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
