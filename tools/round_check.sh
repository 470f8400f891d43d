#!/bin/bash
# Round-end check of the committed tree in one GPU call: every -m gpu test, smoke(), the default bench line
# (bf16 C2) and the fp32x3 C2 line with its rocprof summary.  Usage: tools/round_check.sh TAG
TAG=${1:-r03final}
OUT=gpurun_out/$TAG
bash tools/gpu_step.sh $OUT \
  "tests:::900:::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:::200:::python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:::300:::python -u bench.py" \
  "c4:::300:::python -u bench.py --config c4" \
  "x3prof:::900:::bash tools/prof_x3.sh ${TAG}_x3 fp32x3"
