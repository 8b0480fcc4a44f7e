set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_kmeans_gpu.py tests/test_kmeans_cosine.py > gpurun_out/kc3_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/kc3_tests.log | head -20; tail -30 gpurun_out/kc3_tests.log; exit 1; }
tail -1 gpurun_out/kc3_tests.log
for v in 0 1 0 1; do
  CYC_KMEANS_CANDS3=$v timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/kc3_$v.json 2> gpurun_out/kc3_$v.err || { echo BENCH FAIL; tail -20 gpurun_out/kc3_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/kc3_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('cands3=$v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(x,3) for k,x in {**r['kernels_ms_per_step'], **r.get('diag_kernels_ms_per_step', {})}.items()}, r.get('screen_tiers'))"
done
