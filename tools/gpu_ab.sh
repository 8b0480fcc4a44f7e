# A/B of an env knob ($KNOB=1 vs unset) on one bench workload ($WL): the GPU
# tests in $TESTS with the knob on, then interleaved bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KNOB=${KNOB:?}; WL=${WL:-kmeans}; TESTS=${TESTS:-tests/test_kmeans_gpu.py}
env $KNOB=1 timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export $KNOB=1; else unset $KNOB; fi
  timeout -k 10 300 python -u bench.py --workload $WL --cpu-seconds 0 > gpurun_out/bench_ab$v.json 2> gpurun_out/bench_ab$v.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_ab$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_ab$v.json'));r=d['roofline'];print('$KNOB=$v', round(d['ms_per_step'],2), 'ms', {k: round(x,3) for k,x in r['kernels_ms_per_step'].items()}, round(r['frac'],3))"
done
