# r05c: SCD-only v5 parity; three-way C2 agreement (bf16 / fp32x3 / exact fp32); CPU full-utterance validation;
# TCC hit/miss + HBM bytes of v5 / v10 at the level-0 Conv_0 and cat Conv_0 shapes
O=$PWD/gpurun_out/r05c
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c2_path.py tests/test_gpu_h10.py -x -q --timeout 300 --timeout-method thread" \
 "agree3:::600:::cd $R && python -u tools/agree3.py --out $O/agree3.json" \
 "tcc:::400:::cd $R && bash tools/pmc_tcc.sh $O/tcc 5,10 0,1" \
 "cpufull:::600:::cd $R && python -u bench.py --cpu-full $O/cpu_full_n30.json"
