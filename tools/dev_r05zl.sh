# r05zl: last check of the final tree: GPU suite + smoke
O=$PWD/gpurun_out/r05zl
R=$GRAFT_REPO_ROOT
bash tools/gpu_step.sh $O \
 "tests:::600:::cd $R && python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:::200:::cd $R && python -u -c 'import __graft_entry__ as g; g.smoke()'"
