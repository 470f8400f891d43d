#!/bin/bash
# Round-end check on one GPU box: GPU tests, smoke, the default bench line, a rocprof kernel summary of the fp16 C2
# line (only the timed steps: bench.py's roctx region under --selected-regions), and FETCH_SIZE / WRITE_SIZE passes
# for the halo-GEMM traffic per launch.
# Usage: tools/round_final.sh TAG   (outputs under gpurun_out/TAG; each step under its own time limit)
TAG=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
bash "$ROOT/tools/gpu_step.sh" "$O" \
  "tests:::600:::cd $ROOT && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:::200:::cd $ROOT && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:::300:::cd $ROOT && python -u bench.py" \
  "trace:::400:::cd /tmp && export TMPDIR=/tmp && SNRSE_ROCTX=1 rocprofv3 --kernel-trace --marker-trace --stats --selected-regions --output-format csv -d $O/trace -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe > $O/bench_traced.json && rm -f $O/trace/run_kernel_trace.csv" \
  "fetch:::300:::cd /tmp && export TMPDIR=/tmp && timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity-mode --no-parity" \
  "write:::300:::cd /tmp && export TMPDIR=/tmp && timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity-mode --no-parity" \
  "tracex3:::400:::cd /tmp && export TMPDIR=/tmp && SNRSE_ROCTX=1 rocprofv3 --kernel-trace --marker-trace --stats --selected-regions --output-format csv -d $O/tracex3 -o run -- python3 $ROOT/bench.py --dtype fp32x3 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O/bench_x3_traced.json && rm -f $O/tracex3/run_kernel_trace.csv" \
  "traffic:::120:::cd $ROOT && for k in conv_halo5_kernel; do python3 tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv \$k $O/pmc_traffic_\$k.json || exit 1; done && rm -rf $O/fetch $O/write"
