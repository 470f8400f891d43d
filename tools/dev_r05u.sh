# r05u: the tap-partials pyramid head (conv_head_part_kernel, option head_part): head tests, head micro-bench
# (both forms interleaved; and the 2-workgroups-per-CU build), then an ABAB of the bf16 line with head_part 1 / 0
O=$PWD/gpurun_out/r05u
R=$GRAFT_REPO_ROOT
V=$R/snr-aligned_diffse_amd/lib/var_hp2/libsnrse_hip.so
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "headb:::200:::cd $R && python -u tools/head_bench.py > $O/head_bench.jsonl" \
 "headb2:::200:::cd $R && SNRSE_LIB=$V python -u tools/head_bench.py > $O/head_bench_minb2.jsonl" \
 "bf_p1a:::200:::cd $R && $L > $O/bf_p1a.json" \
 "bf_p0a:::200:::cd $R && SNRSE_OPTS=head_part=0 $L > $O/bf_p0a.json" \
 "bf_p1b:::200:::cd $R && $L > $O/bf_p1b.json" \
 "bf_p0b:::200:::cd $R && SNRSE_OPTS=head_part=0 $L > $O/bf_p0b.json"
