# One rocprofv3 --pmc pass (its own run, no tracing domains) over a short
# bench.py run.  usage: bash tools/pmc_pass.sh <tag> "<counters>" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; CTRS=$2; shift 2
export TMPDIR=/tmp
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace -T -d $OUT -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 "$@" > $OUT/log.txt 2>&1
