# r05z: compile-time epilogue flags for the fp32x3 halo GEMM's pair schedule (option h5_specialise, which in the
# fp32x3 mode only selects these): GPU suite, then an ABAB of the fp32x3 line with h5_specialise 1 / 0
O=$PWD/gpurun_out/r05z
R=$GRAFT_REPO_ROOT
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "x3_s1a:::200:::cd $R && $X > $O/x3_s1a.json" \
 "x3_s0a:::200:::cd $R && SNRSE_OPTS=h5_specialise=0 $X --no-parity > $O/x3_s0a.json" \
 "x3_s1b:::200:::cd $R && $X --no-parity > $O/x3_s1b.json" \
 "x3_s0b:::200:::cd $R && SNRSE_OPTS=h5_specialise=0 $X --no-parity > $O/x3_s0b.json"
