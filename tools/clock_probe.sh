#!/bin/bash
# Effective shader clock of the v10 halo GEMM per build (MI355X_MICROARCH.md DVFS note: GRBM_GUI_ACTIVE / 8 / kernel
# time): one rocprofv3 pass with GRBM_GUI_ACTIVE + kernel trace per library.  Usage: tools/clock_probe.sh OUTDIR lib...
set -e
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename "$(dirname "$L")")
  SNRSE_LIB="$ROOT/$L" timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv \
    -d "$OUT/$n" -o run -- python3 "$ROOT/tools/conv_bench.py" --variants 10 --shapes 0 --reps 3 --rounds 1 --gn > "$OUT/$n.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*/"))):
    n = os.path.basename(d.rstrip("/"))
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        continue
    g = [float(r["Counter_Value"]) for r in csv.DictReader(open(cc[0])) if "conv_halo10" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(kt[0])) if "conv_halo10" in r["Kernel_Name"]]
    if g and t:
        gm, tm = sum(g) / len(g), sum(t) / len(t)
        res[n] = {"grbm_gui_active": gm, "kernel_us": tm / 1e3, "clock_ghz": gm / 8 / tm}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "clocks.json"), "w"), indent=1)
PY
