# A/B of a KMeans screen knob (env var $KNOB=1 vs unset): KMeans GPU tests
# with the knob on, then interleaved bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KNOB=${KNOB:-CYC_KM2_PF}
env $KNOB=1 timeout -k 10 400 python -u -m pytest tests/test_kmeans_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_km_ab.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/pytest_km_ab.log; exit 1; }
tail -1 gpurun_out/pytest_km_ab.log
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export $KNOB=1; else unset $KNOB; fi
  timeout -k 10 300 python -u bench.py --workload kmeans --cpu-seconds 0 > gpurun_out/bench_km_ab$v.json 2> gpurun_out/bench_km_ab$v.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_km_ab$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_km_ab$v.json'));r=d['roofline'];print('$KNOB=$v', round(d['ms_per_step'],2), 'ms', {k: round(x,3) for k,x in r['kernels_ms_per_step'].items()}, round(r['frac'],3))"
done
