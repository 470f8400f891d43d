# r05zi: the halo GEMM residual convs' residual vectors requested early (half 0 before the final drain, half 1 before
# half 0's passes): GPU suite, ABAB of the bf16 line against HEAD's library (var_base)
O=$PWD/gpurun_out/r05zi
R=$GRAFT_REPO_ROOT
B=$R/snr-aligned_diffse_amd/lib/var_base/libsnrse_hip.so
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bf_new1:::200:::cd $R && $L > $O/bf_new1.json" \
 "bf_base1:::200:::cd $R && SNRSE_LIB=$B $L > $O/bf_base1.json" \
 "bf_new2:::200:::cd $R && $L > $O/bf_new2.json" \
 "bf_base2:::200:::cd $R && SNRSE_LIB=$B $L > $O/bf_base2.json"
