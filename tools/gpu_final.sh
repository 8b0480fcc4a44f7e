# Round-end validation: every GPU test, the four bench lines (with CPU
# baselines), and rocprofv3 stats + PMC passes for the given workloads.
# usage: bash tools/gpu_final.sh [workload to profile ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for w in kmeans gramian lr_multi lr_sparse; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],3), (d['cpu_baseline'] or {}).get('value'))"
done
for w in "$@"; do
  case $w in kmeans) st=3; wu=2;; gramian) st=2; wu=1;; *) st=3; wu=1;; esac
  bash tools/prof.sh prof_$w --workload $w --steps $st --warmup $wu || { echo PROF $w FAIL; exit 1; }
done
echo ALLDONE
