# r05f: GPU tests of the round-5 kernels; three-way C2 agreement; v5 A/B (round 4 / SCD / SCD + waitcnt-model fix);
# fp32x3 pair schedule A/B; pyramid-head prefetch A/B; the default bench line
O=$PWD/gpurun_out/r05f
R=$GRAFT_REPO_ROOT
L=$R/snr-aligned_diffse_amd/lib
bash tools/gpu_step.sh $O \
 "tests:::400:::cd $R && python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread" \
 "agree3:::300:::cd $R && python -u tools/agree3.py --out $O/agree3.json" \
 "v5ab:::400:::cd $R && bash tools/ab_conv.sh $O/v5ab 2 0,1,2,3,4,7 $L/var_head/libsnrse_hip.so $L/var_scd/libsnrse_hip.so default" \
 "x3pair:::200:::cd $R && python3 tools/x3_bench.py --tiles 0 --exact 0 --gn 1 --spread 2,1,2,1 --reps 10" \
 "headab:::200:::cd $R && for lib in $L/var_head/libsnrse_hip.so $L/libsnrse_hip.so $L/var_hd3/libsnrse_hip.so $L/var_head/libsnrse_hip.so $L/libsnrse_hip.so $L/var_hd3/libsnrse_hip.so; do echo lib \$lib; SNRSE_LIB=\$lib python3 tools/head_bench.py || exit 1; done" \
 "bench:::300:::cd $R && python -u bench.py > $O/bench.json"
