# r05q: persistent fp32x3 halo GEMM (variant library lib/var_x3p, option x3_persist): parity under persistence,
# then interleaved per-shape timings default / var persist 0 / var persist 1
O=$PWD/gpurun_out/r05q
R=$GRAFT_REPO_ROOT
V=$R/snr-aligned_diffse_amd/lib/var_x3p/libsnrse_hip.so
B="python3 -u tools/x3_bench.py --tiles 0 --exact 0 --gn 1 --spread 2 --reps 10"
bash tools/gpu_step.sh $O \
 "x3tests:::300:::cd $R && SNRSE_LIB=$V SNRSE_OPTS=x3_persist=1 python -u -m pytest tests/test_gpu_x3.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "a1:::150:::cd $R && $B > $O/a1_default.jsonl" \
 "b1:::150:::cd $R && SNRSE_LIB=$V SNRSE_OPTS=x3_persist=0 $B > $O/b1_var0.jsonl" \
 "c1:::150:::cd $R && SNRSE_LIB=$V SNRSE_OPTS=x3_persist=1 $B > $O/c1_var1.jsonl" \
 "a2:::150:::cd $R && $B > $O/a2_default.jsonl" \
 "b2:::150:::cd $R && SNRSE_LIB=$V SNRSE_OPTS=x3_persist=0 $B > $O/b2_var0.jsonl" \
 "c2:::150:::cd $R && SNRSE_LIB=$V SNRSE_OPTS=x3_persist=1 $B > $O/c2_var1.jsonl"
