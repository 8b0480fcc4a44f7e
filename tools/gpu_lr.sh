# Logistic-aggregator loop on the GPU box: the logistic GPU tests, then the
# multinomial and sparse bench lines (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_logistic_gpu.py tests/test_lr_fit.py ${LR_TESTS:-} -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { echo LR TESTS FAIL; grep -E "FAILED|Error|error" gpurun_out/lr_tests.log | head -20; tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
for w in ${LR_BENCH:-lr_multi}; do
timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 3 --cpu-seconds 0 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
python - "$w" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], round(d["value"] / 1e6, 1), "M rows/s", round(d["ms_per_step"], 3), "ms", r["kernel"], round(r["frac"], 4), {k: round(v, 3) for k, v in r["kernels_ms_per_step"].items()})
PY
done
echo ALLDONE
