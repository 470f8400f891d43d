# r05ze part 1: final round check of the committed code: GPU suite, smoke, default line, rocprof kernel stats (bf16)
O=$PWD/gpurun_out/r05ze
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
  "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:::300:::cd $R && python -u bench.py > $O/bench.json" \
  "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe > $O/bench_traced.json && rm -f $O/trace/run_kernel_trace.csv"
