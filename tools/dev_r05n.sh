# r05n: split-K finalize with batched partial loads + the two-chunk-ahead head (re-applied): GPU suite, smoke,
# head micro-bench, line, traced line
O=$PWD/gpurun_out/r05n
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::700:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::300:::cd $R && python -u bench.py --no-cpu-baseline > $O/bench.json" \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv" \
 "tracex3:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/tracex3 -o run -- python3 $R/bench.py --dtype fp32x3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-parity > $O/bench_x3_traced.json && python3 $R/tools/dispatch_shapes.py $O/tracex3/run_kernel_trace.csv > $O/dispatch_shapes_x3.jsonl && rm -f $O/tracex3/run_kernel_trace.csv"
