# r05p: fp32x3 mode with split-bf16 attention core + projections: GPU suite, smoke, x3 line, x3 traced dispatch shapes
O=$PWD/gpurun_out/r05p
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::700:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "x3line:::300:::cd $R && python -u bench.py --dtype fp32x3 --steps 3 --no-cpu-baseline > $O/x3line.json" \
 "tracex3:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/tracex3 -o run -- python3 $R/bench.py --dtype fp32x3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-parity > $O/bench_x3_traced.json && python3 $R/tools/dispatch_shapes.py $O/tracex3/run_kernel_trace.csv > $O/dispatch_shapes_x3.jsonl && rm -f $O/tracex3/run_kernel_trace.csv"
