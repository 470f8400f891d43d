O=$PWD/gpurun_out/r05a
bash tools/gpu_step.sh $O \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $GRAFT_REPO_ROOT/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv" \
 "cbench:::300:::cd $GRAFT_REPO_ROOT && python3 tools/conv_bench.py --variants 5,10 --rounds 2 --reps 10 --gn --shapes 0,2,7,8"
