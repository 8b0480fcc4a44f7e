#!/bin/bash
# One PMC pass (waves launched, wave / busy cycles, instruction mix) over a
# bench workload, filtered to the kernels matching a regex.
# usage: tools/pmc_waves.sh <tag> <regex> [bench args]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
TAG=$1; RX=$2; shift 2
OUT=$R/gpurun_out/pmcw_$TAG
mkdir -p $OUT
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex "$RX" -d $OUT/p -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 "$@" > $OUT/p.log 2>&1 || { echo "pass failed"; tail -5 $OUT/p.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        agg[(name.split("(")[0][-60:], r["Counter_Name"])].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    for k in sorted(agg):
        v = agg[k]
        line = f"{k[0]:60s} {k[1]:20s} {sum(v)/len(v):14.4e} (n={len(v)})"
        print(line); fo.write(line + "\n")
PY
find $OUT -name '*.csv' -size +20M -delete
