# r05zg: non-temporal stores in the row-strip resampler (option resample_nt 1; the fp32x3 mode writes 4.3 GB per
# level-0 up launch) against the default, ABAB on the fp32x3 line, one pair on the bf16 line
O=$PWD/gpurun_out/r05zg
R=$GRAFT_REPO_ROOT
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline --no-parity"
bash tools/gpu_step.sh $O \
 "xd1:::200:::cd $R && $X > $O/xd1.json" \
 "xn1:::200:::cd $R && SNRSE_OPTS=resample_nt=1 $X > $O/xn1.json" \
 "xd2:::200:::cd $R && $X > $O/xd2.json" \
 "xn2:::200:::cd $R && SNRSE_OPTS=resample_nt=1 $X > $O/xn2.json" \
 "d1:::200:::cd $R && $L > $O/d1.json" \
 "n1:::200:::cd $R && SNRSE_OPTS=resample_nt=1 $L > $O/n1.json"
