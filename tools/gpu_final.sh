# Round-end validation: every GPU test + smoke (PART=tests), the four bench
# lines with CPU baselines (PART=bench), or both (default).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PART=${PART:-all}
if [ $PART != bench ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
fi
if [ $PART != tests ]; then
for w in ${WL:-kmeans gramian lr_multi lr_sparse}; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],3), (d['cpu_baseline'] or {}).get('value'))"
done
fi
echo ALLDONE
