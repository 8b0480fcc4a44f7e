# usage: bash tools/gpu_tests.sh <pytest args...>  (GPU-marked tests, one process)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { echo PYTEST FAIL; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_sel.log | head -30; tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -3 gpurun_out/pytest_sel.log
