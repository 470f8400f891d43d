# r05zc: the fp32x3 halo GEMM's epilogue bias + temb staged in LDS at the tile start (no round trip after the main
# loop): GPU suite, ABAB of the fp32x3 line against HEAD's library (var_base)
O=$PWD/gpurun_out/r05zc
R=$GRAFT_REPO_ROOT
B=$R/snr-aligned_diffse_amd/lib/var_base/libsnrse_hip.so
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "x3_new1:::200:::cd $R && $X > $O/x3_new1.json" \
 "x3_base1:::200:::cd $R && SNRSE_LIB=$B $X --no-parity > $O/x3_base1.json" \
 "x3_new2:::200:::cd $R && $X --no-parity > $O/x3_new2.json" \
 "x3_base2:::200:::cd $R && SNRSE_LIB=$B $X --no-parity > $O/x3_base2.json"
