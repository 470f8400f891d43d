# r05zf: non-temporal halo-GEMM output stores from 128 MB of output (epi_nt_mb 128: the level-1 256 MiB outputs too)
# against the default 256, ABAB on the bf16 line and one pair on the fp32x3 line
O=$PWD/gpurun_out/r05zf
R=$GRAFT_REPO_ROOT
L="python -u bench.py --no-cpu-baseline --no-parity-mode --steps 10 --warmup 3"
X="python -u bench.py --dtype fp32x3 --steps 3 --warmup 2 --no-cpu-baseline --no-parity"
bash tools/gpu_step.sh $O \
 "d1:::200:::cd $R && $L > $O/d1.json" \
 "n1:::200:::cd $R && SNRSE_OPTS=epi_nt_mb=128 $L > $O/n1.json" \
 "d2:::200:::cd $R && $L > $O/d2.json" \
 "n2:::200:::cd $R && SNRSE_OPTS=epi_nt_mb=128 $L > $O/n2.json" \
 "xd:::200:::cd $R && $X > $O/xd.json" \
 "xn:::200:::cd $R && SNRSE_OPTS=epi_nt_mb=128 $X > $O/xn.json"
