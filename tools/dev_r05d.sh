# r05d: three-way C2 agreement; v5 A/B: round-4 code (var_head) vs the committed SCD code (default) vs the unrolled
# chunk loop (var_unr); per-shape TCC counters of v5 / v10 (separate shapes)
O=$PWD/gpurun_out/r05d
R=$GRAFT_REPO_ROOT
L=$R/snr-aligned_diffse_amd/lib
bash tools/gpu_step.sh $O \
 "agree3:::600:::cd $R && python -u tools/agree3.py --out $O/agree3.json" \
 "ab:::900:::cd $R && bash tools/ab_conv.sh $O/ab 2 0,1,2,3,4,7 $L/var_head/libsnrse_hip.so default $L/var_unr/libsnrse_hip.so" \
 "tcc0:::300:::cd $R && bash tools/pmc_tcc.sh $O/tcc0 5,10 0" \
 "tcc1:::300:::cd $R && bash tools/pmc_tcc.sh $O/tcc1 5,10 1" || exit 1
cd $R && for lib in $L/var_head/libsnrse_hip.so $L/libsnrse_hip.so $L/var_hd3/libsnrse_hip.so $L/var_head/libsnrse_hip.so $L/libsnrse_hip.so $L/var_hd3/libsnrse_hip.so; do echo "lib $lib"; SNRSE_LIB=$lib timeout -k 10 120 python3 tools/head_bench.py || exit 1; done > $O/head_ab.log 2>&1 || exit 1
cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
