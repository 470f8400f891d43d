# r05s: GroupNorm apply with the first input batch before the fold, two-pixel split-K finalize steps:
# GPU suite, smoke, line, traced line (+ the same traced with option head_small 2: the small head at level 4 too)
O=$PWD/gpurun_out/r05s
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::300:::cd $R && python -u bench.py --no-cpu-baseline > $O/bench.json" \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv" \
 "traceh2:::400:::cd /tmp && export TMPDIR=/tmp && SNRSE_OPTS=head_small=2 rocprofv3 --kernel-trace --output-format csv -d $O/traceh2 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced_h2.json && python3 $R/tools/dispatch_shapes.py $O/traceh2/run_kernel_trace.csv > $O/dispatch_shapes_h2.jsonl && rm -f $O/traceh2/run_kernel_trace.csv"
