# r05x: round check of the committed code (epilogue prefetch, tap-partials head): GPU suite, smoke, default line, x3 line
O=$PWD/gpurun_out/r05x
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
  "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:::300:::cd $R && python -u bench.py > $O/bench.json" \
  "x3line:::300:::cd $R && python -u bench.py --dtype fp32x3 --steps 3 --no-cpu-baseline > $O/x3line.json"
