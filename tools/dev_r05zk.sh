# r05zk: LLVM machine-scheduler strategies for the whole library (-mllvm -amdgpu-sched-strategy=max-ilp /
# max-memory-clause; tools/build_variant.py) against the default, interleaved on the bf16 line
O=$PWD/gpurun_out/r05zk
R=$GRAFT_REPO_ROOT
V=$R/snr-aligned_diffse_amd/lib
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
bash tools/gpu_step.sh $O \
 "b1:::200:::cd $R && $L > $O/b1.json" \
 "i1:::200:::cd $R && SNRSE_LIB=$V/var_ilp/libsnrse_hip.so $L > $O/i1.json" \
 "m1:::200:::cd $R && SNRSE_LIB=$V/var_mclause/libsnrse_hip.so $L > $O/m1.json" \
 "b2:::200:::cd $R && $L > $O/b2.json" \
 "i2:::200:::cd $R && SNRSE_LIB=$V/var_ilp/libsnrse_hip.so $L > $O/i2.json" \
 "m2:::200:::cd $R && SNRSE_LIB=$V/var_mclause/libsnrse_hip.so $L > $O/m2.json"
