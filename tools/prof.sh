#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement").
# usage: bash tools_prof.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
export TMPDIR=/tmp
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d $OUT/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d $OUT/pmc_write -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/pmc_write.log 2>&1 || exit $?
