# r05b: v5 shortcut phases as LDS-DMA (option h5_sc): parity tests, per-shape A/B, whole-line ABAB
O=$PWD/gpurun_out/r05b
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c2_path.py -x -q --timeout 300 --timeout-method thread" \
 "cbench:::400:::cd $R && python3 tools/conv_bench.py --option h5_sc --variants 1,0 --rounds 3 --reps 10 --gn --shapes 2,7,8,9,10,11" \
 "benchB0:::300:::cd $R && SNRSE_OPTS=h5_sc=0 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/bench_sc0_a.json" \
 "benchB1:::300:::cd $R && python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/bench_sc1_a.json" \
 "benchB0b:::300:::cd $R && SNRSE_OPTS=h5_sc=0 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/bench_sc0_b.json" \
 "benchB1b:::300:::cd $R && python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/bench_sc1_b.json"
