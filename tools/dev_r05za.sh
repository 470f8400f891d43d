# r05za: fp32x3 compile-time epilogues also for the Combine convs and the GroupNorm-free (post-resampler) convs: GPU suite,
# ABAB of the fp32x3 line with h5_specialise 1 / 0, one traced fp32x3 step for the per-dispatch table
O=$PWD/gpurun_out/r05za
R=$GRAFT_REPO_ROOT
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "x3_s1a:::200:::cd $R && $X > $O/x3_s1a.json" \
 "x3_s0a:::200:::cd $R && SNRSE_OPTS=h5_specialise=0 $X --no-parity > $O/x3_s0a.json" \
 "x3_s1b:::200:::cd $R && $X --no-parity > $O/x3_s1b.json" \
 "x3_s0b:::200:::cd $R && SNRSE_OPTS=h5_specialise=0 $X --no-parity > $O/x3_s0b.json"
bash tools/gpu_step.sh $O \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --dtype fp32x3 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-parity > $O/x3_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/x3_dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv"
