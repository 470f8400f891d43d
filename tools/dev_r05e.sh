# r05e: fp32x3 halo GEMM (conv_x3h_kernel) ablations + SQ counters; v5 waitcnt-model fix (var_vm) A/B; CPU validation
O=$PWD/gpurun_out/r05e
R=$GRAFT_REPO_ROOT
L=$R/snr-aligned_diffse_amd/lib
bash tools/gpu_step.sh $O \
 "x3ab:::900:::cd $R && bash tools/ab_x3.sh $O/x3ab 2 default $L/var_x3noepi/libsnrse_hip.so $L/var_x3noxf/libsnrse_hip.so $L/var_x3nohalo/libsnrse_hip.so $L/var_x3bar3/libsnrse_hip.so $L/var_x3mfma/libsnrse_hip.so" \
 "x3sq:::300:::cd $R && bash tools/pmc_x3.sh $O/x3sq 0" \
 "vmab:::600:::cd $R && bash tools/ab_conv.sh $O/vmab 2 0,1,2,3,4,7 default $L/var_vm/libsnrse_hip.so" \
 "cpufull:::600:::cd $R && python -u bench.py --cpu-full $O/cpu_full_n30.json"
