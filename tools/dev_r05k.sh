# r05k: tail launches round 2 (one-launch GroupNorm apply on the small levels, 64 x 256 LDS-DMA GEMM tiles):
# full GPU suite, smoke, line A/B/A on option glds_bm64, traced line with per-dispatch shapes
O=$PWD/gpurun_out/r05k
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::700:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "benchA:::300:::cd $R && python -u bench.py --no-cpu-baseline > $O/benchA.json" \
 "benchB:::300:::cd $R && SNRSE_OPTS=glds_bm64=0 python -u bench.py --no-cpu-baseline --no-parity-mode > $O/benchB.json" \
 "benchA2:::300:::cd $R && python -u bench.py --no-cpu-baseline --no-parity-mode > $O/benchA2.json" \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv"
