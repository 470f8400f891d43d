# r05m: pyramid head with two-chunk-ahead halo loads, MFMA time-embedding dense, 16 fold blocks per image
O=$PWD/gpurun_out/r05m
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::700:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "head:::120:::cd $R && python -u tools/head_bench.py > $O/head_bench.jsonl" \
 "bench:::300:::cd $R && python -u bench.py --no-cpu-baseline > $O/bench.json" \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv"
