#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at a crash / timeout / fault (exit codes
# 124, 134, 137, 139 or a negative signal), continue after an ordinary test failure (exit 1).
# Usage: tools/gpu_step.sh OUTDIR "name1:::limit1:::cmd1" "name2:::limit2:::cmd2" ...
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:::*}; rest=${spec#*:::}; lim=${rest%%:::*}; cmd=${rest#*:::}
  echo "[gpu_step] $name (limit ${lim}s): $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[gpu_step] $name rc=$rc" | tee -a "$OUT/steps.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "[gpu_step] stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"; exit $rc ;;
  esac
done
