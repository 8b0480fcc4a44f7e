#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement").
# usage: bash tools/prof.sh <tag> [bench args...]
# Three separate rocprofv3 runs: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE each in its own --pmc pass (MI355X_MICROARCH.md, HBM section).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
export TMPDIR=/tmp
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/pmc_write.log 2>&1 || exit $?
# With SUMMARY=<rows>:<iterations>, summarise on the box into
# $OUT/summary_{pmc.json,kernel_stats.csv} and drop the raw per-dispatch
# CSVs (they can exceed what gpurun copies back).
if [ -n "$SUMMARY" ]; then
  python3 $R/tools/pmc_summary.py $OUT $OUT/summary ${SUMMARY%%:*} ${SUMMARY##*:} > $OUT/summary.log 2>&1 || exit $?
  find $OUT -name '*.csv' ! -name 'summary_*' ! -name 'run_kernel_stats.csv' -delete
fi
