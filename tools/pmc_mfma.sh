#!/bin/bash
# MFMA-busy / issue PMC passes (separate rocprofv3 runs) over one bench
# workload, kernels filtered by a regex.
# usage: tools/pmc_mfma.sh <tag> <kernel regex> [bench args]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
TAG=$1; RX=$2; shift 2
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$RX" -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --steps 2 --warmup 1 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        nm = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0].replace("void ", "").split("::")[-1][:60]
        agg[(nm, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k[0]:60s} {k[1]:28s} {sum(v)/len(v):16.4e} (n={len(v)})")
PY
