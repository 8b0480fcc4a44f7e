# Iteration run: the GPU test files in TESTS (default: all; "none" skips),
# then (PROF=1) the round-2 profiles of WL, then one bench line per workload
# in WL (after the profiles, so their PMC traffic is the one reported).
# Stops at the first crash-like exit (not at a plain test failure).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$TESTS" != none ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 600 --timeout-method thread --durations=10 > gpurun_out/iter_tests.log 2>&1
rc=$?
grep -E "FAILED|Error" gpurun_out/iter_tests.log | head -5
tail -3 gpurun_out/iter_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "$PROF" = 1 ]; then WL="$WL" bash tools/gpu_prof_r02.sh || exit 1; fi
for w in $WL; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];print('$w', round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['frac'],3), {k: round(v,3) for k,v in r.get('kernels_ms_per_step',{}).items()}, {k: v for k,v in r.items() if k.startswith('rows_')})"
done
echo ALLDONE
