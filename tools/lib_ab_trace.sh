#!/bin/bash
# In-situ A/B of two library builds: rocprofv3 --kernel-trace --stats over a short C2 bench (N=2) for
# each, alternating A B A B; prints per-run the listed kernels' mean durations and the sum of all kernels.
# Usage: tools/lib_ab_trace.sh OUTTAG B "kernel substr,..."   (A = the default in-tree library and options;
#        B = a library path relative to the repo, or opts:NAME=V[,NAME=V] for SNRSE_OPTS on the default one)
set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/$1
BSPEC=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
I=0
for V in A B A B; do
  I=$((I+1))
  unset SNRSE_LIB SNRSE_OPTS
  if [ $V = B ]; then
    case $BSPEC in
      opts:*) export SNRSE_OPTS=${BSPEC#opts:} ;;
      *) export SNRSE_LIB=$ROOT/$BSPEC ;;
    esac
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$I -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --N 2 --no-cpu-baseline --no-probe > $OUT/b$I.log 2>&1
  python3 - $OUT/t$I/run_kernel_stats.csv $V "$3" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
out = {'lib': sys.argv[2], 'all_kernels_ms': tot / 1e6}
for sub in sys.argv[3].split(','):
    for r in rows:
        if sub in r['Name']:
            out[sub + '_us'] = float(r['AverageNs']) / 1e3
print(out)
PY
  rm -f $OUT/t$I/run_kernel_trace.csv
done
