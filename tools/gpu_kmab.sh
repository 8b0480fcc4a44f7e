set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CYC_KM32_W8=1 timeout -k 10 400 python -u -m pytest tests/test_kmeans_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_km_w8.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/pytest_km_w8.log; exit 1; }
tail -1 gpurun_out/pytest_km_w8.log
for v in 4 8 4 8; do
  if [ $v = 8 ]; then export CYC_KM32_W8=1; else unset CYC_KM32_W8; fi
  timeout -k 10 300 python -u bench.py --workload kmeans --cpu-seconds 0 > gpurun_out/bench_km_w$v.json 2> gpurun_out/bench_km_w$v.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_km_w$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_km_w$v.json'));r=d['roofline'];print('W$v', round(d['ms_per_step'],2), 'ms', round(r['avg_launch_ms'],3), round(r['frac'],3))"
done
