# Bench-size parity tests (large shards), then the bench lines of the four workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gramian_gpu.py tests/test_logistic_gpu.py -x -v --timeout 600 --timeout-method thread --durations=6 -k "bench_shard" > gpurun_out/big_tests.log 2>&1 || { echo BIG TESTS FAIL; grep -E "FAILED|Error" gpurun_out/big_tests.log | head; tail -40 gpurun_out/big_tests.log; exit 1; }
grep -E "passed|PASSED|slowest" -A0 gpurun_out/big_tests.log | tail -5
for w in ${WL:-kmeans gramian lr_multi lr_sparse}; do
  timeout -k 10 600 python -u bench.py --workload $w ${CPU:+--cpu-seconds $CPU} > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];print('$w', round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['frac'],3), {k: round(v,2) for k,v in r['kernels_ms_per_step'].items()}, (d['cpu_baseline'] or {}).get('value'))"
done
