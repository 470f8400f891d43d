# r05i: full GPU suite, smoke, the default line and the fp32x3 line on the committed code
O=$PWD/gpurun_out/r05i
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::700:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:::300:::cd $R && python -u bench.py > $O/bench.json" \
 "x3line:::300:::cd $R && python -u bench.py --dtype fp32x3 --steps 3 --no-cpu-baseline > $O/x3line.json"
