# r05t: GEMM epilogues request the residual / Combine inputs passes ahead (no per-pass HBM round trip that
# also drained the earlier stores): GPU suite on the new library, then interleaved A/B of the bf16 and fp32x3
# lines against HEAD's library (var_base), then one traced bf16 step for the per-dispatch table
O=$PWD/gpurun_out/r05t
R=$GRAFT_REPO_ROOT
B=$R/snr-aligned_diffse_amd/lib/var_base/libsnrse_hip.so
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline --no-parity"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bf_new1:::200:::cd $R && $L > $O/bf_new1.json" \
 "bf_base1:::200:::cd $R && SNRSE_LIB=$B $L > $O/bf_base1.json" \
 "bf_new2:::200:::cd $R && $L > $O/bf_new2.json" \
 "bf_base2:::200:::cd $R && SNRSE_LIB=$B $L > $O/bf_base2.json" \
 "x3_new1:::200:::cd $R && $X > $O/x3_new1.json" \
 "x3_base1:::200:::cd $R && SNRSE_LIB=$B $X > $O/x3_base1.json" \
 "x3_new2:::200:::cd $R && $X > $O/x3_new2.json" \
 "x3_base2:::200:::cd $R && SNRSE_LIB=$B $X > $O/x3_base2.json" \
 "trace:::400:::cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity-mode --no-probe --no-parity > $O/bench_traced.json && python3 $R/tools/dispatch_shapes.py $O/trace/run_kernel_trace.csv > $O/dispatch_shapes.jsonl && rm -f $O/trace/run_kernel_trace.csv"
