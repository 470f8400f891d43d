# r05g: fp32x3 halo GEMM ablations + SQ counters; TCC hit / miss of v5 / v10; the fp32x3 line with the pair schedule;
# CPU full-utterance validation
O=$PWD/gpurun_out/r05g
R=$GRAFT_REPO_ROOT
L=$R/snr-aligned_diffse_amd/lib
bash tools/gpu_step.sh $O \
 "tests:::500:::cd $R && python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_c2_path.py tests/test_gpu_kernels.py -k 'x3 or c2 or head or halo' -x -q --timeout 300 --timeout-method thread" \
 "x3ab:::500:::cd $R && bash tools/ab_x3.sh $O/x3ab 1 default $L/var_x3noepi/libsnrse_hip.so $L/var_x3noxf/libsnrse_hip.so $L/var_x3nohalo/libsnrse_hip.so $L/var_x3bar3/libsnrse_hip.so $L/var_x3mfma/libsnrse_hip.so" \
 "x3sq:::200:::cd $R && bash tools/pmc_x3.sh $O/x3sq 0" \
 "tcc0:::150:::cd $R && bash tools/pmc_tcc.sh $O/tcc0 5,10 0" \
 "tcc1:::150:::cd $R && bash tools/pmc_tcc.sh $O/tcc1 5,10 1" \
 "cpufull:::400:::cd $R && python -u bench.py --cpu-full $O/cpu_full_n30.json"
