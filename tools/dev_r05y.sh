# r05y: the two-lane sampler (--streams 2, each lane a half batch on its own HIP stream; --stagger 1: the second
# lane half an NFE behind) against one lane, interleaved
O=$PWD/gpurun_out/r05y
R=$GRAFT_REPO_ROOT
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
bash tools/gpu_step.sh $O \
 "s1a:::200:::cd $R && $L > $O/s1a.json" \
 "s2sa:::200:::cd $R && $L --streams 2 --stagger 1 > $O/s2sa.json" \
 "s2a:::200:::cd $R && $L --streams 2 > $O/s2a.json" \
 "s1b:::200:::cd $R && $L > $O/s1b.json" \
 "s2sb:::200:::cd $R && $L --streams 2 --stagger 1 > $O/s2sb.json" \
 "s2b:::200:::cd $R && $L --streams 2 > $O/s2b.json"
