# r05ze part 2: FETCH_SIZE / WRITE_SIZE passes for the halo-GEMM traffic per launch, the fp32x3 line and its rocprof stats
O=$PWD/gpurun_out/r05ze
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
  "fetch:::300:::cd /tmp && export TMPDIR=/tmp && timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity-mode --no-parity" \
  "write:::300:::cd /tmp && export TMPDIR=/tmp && timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe --no-parity-mode --no-parity" \
  "x3line:::300:::cd $R && python -u bench.py --dtype fp32x3 --steps 3 --no-cpu-baseline > $O/x3line.json" \
  "tracex3:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/tracex3 -o run -- python3 $R/bench.py --dtype fp32x3 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O/bench_x3_traced.json && rm -f $O/tracex3/run_kernel_trace.csv" \
  "traffic:::120:::cd $R && for k in conv_halo5_kernel; do python3 tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv \$k $O/pmc_traffic_\$k.json || exit 1; done && rm -rf $O/fetch $O/write"
