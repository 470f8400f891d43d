# r05h: whole-line A/B of the v10 dispatch (h10 = 2 default / 0 = v5 everywhere / 3) after the v5 changes; v5 vs v10 on
# the level-0 cat Conv_0; the fp32x3 line with the pair schedule
O=$PWD/gpurun_out/r05h
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "cb:::200:::cd $R && python3 tools/conv_bench.py --variants 5,10 --rounds 2 --reps 10 --gn --shapes 1,7" \
 "h2a:::200:::cd $R && python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h2a.json" \
 "h0a:::200:::cd $R && SNRSE_OPTS=h10=0 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h0a.json" \
 "h3a:::200:::cd $R && SNRSE_OPTS=h10=3 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h3a.json" \
 "h2b:::200:::cd $R && python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h2b.json" \
 "h0b:::200:::cd $R && SNRSE_OPTS=h10=0 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h0b.json" \
 "h3b:::200:::cd $R && SNRSE_OPTS=h10=3 python -u bench.py --steps 4 --no-cpu-baseline --no-parity-mode > $O/h3b.json" \
 "x3line:::300:::cd $R && python -u bench.py --dtype fp32x3 --steps 3 --no-cpu-baseline > $O/x3line.json"
