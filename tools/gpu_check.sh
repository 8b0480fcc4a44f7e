# One GPU call: the named test files, then one bench line per workload.
# usage: TESTS="tests/a.py tests/b.py" WLS="pca lr_multi" bash tools/gpu_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/check_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|error" gpurun_out/check_tests.log | head -20; tail -20 gpurun_out/check_tests.log; exit 1; }
  tail -1 gpurun_out/check_tests.log
fi
for w in $WLS; do
  timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 3 --cpu-seconds 0 > gpurun_out/check_$w.json 2> gpurun_out/check_$w.err || { echo BENCH FAIL $w; tail -20 gpurun_out/check_$w.err; exit 1; }
  python - $w <<'PY'
import json, sys
w = sys.argv[1]
d = json.loads(open(f"gpurun_out/check_{w}.json").read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(w, round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"], 2), "ms", r.get("kernel"),
      round(r.get("frac", 0), 4), {k: round(v, 2) for k, v in {**(r.get("kernels_ms_per_step") or {}), **(r.get("diag_kernels_ms_per_step") or {})}.items()},
      r.get("covariance_passes"), r.get("centred_form_ms_per_step"), (d.get("fit") or {}).get("fit_ms"))
PY
done
echo CHECKDONE
