# r05w: the persistent tap-partials head (option head_part 2): head tests, head micro-bench (1 / 2 / 0 interleaved),
# ABAB of the bf16 line with head_part 2 / 1
O=$PWD/gpurun_out/r05w
R=$GRAFT_REPO_ROOT
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
bash tools/gpu_step.sh $O \
 "tests:::300:::cd $R && python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k head" \
 "headb:::200:::cd $R && python -u tools/head_bench.py > $O/head_bench.jsonl" \
 "bf_p2a:::200:::cd $R && SNRSE_OPTS=head_part=2 $L > $O/bf_p2a.json" \
 "bf_p1a:::200:::cd $R && $L > $O/bf_p1a.json" \
 "bf_p2b:::200:::cd $R && SNRSE_OPTS=head_part=2 $L > $O/bf_p2b.json" \
 "bf_p1b:::200:::cd $R && $L > $O/bf_p1b.json"
