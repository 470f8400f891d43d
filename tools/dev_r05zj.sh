# r05zj: SQ counters of the final v5 halo GEMM (conv micro-bench, fused GroupNorm) at the level-0 Conv_0 shape (0) and
# the up-path Conv_1 with the 256-channel cat shortcut (7): one rocprofv3 --pmc pass per counter group
O=$PWD/gpurun_out/r05zj
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "sq0:::600:::cd $R && bash tools/pmc_conv.sh $O/shape0 5 0" \
 "sq7:::600:::cd $R && bash tools/pmc_conv.sh $O/shape7 5 7"
