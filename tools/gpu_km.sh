# KMeans iteration loop on the GPU box: the KMeans GPU tests, then the KMeans
# bench line (no CPU baseline) and the screen tiers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_gpu.py tests/test_kmeans_model_gpu.py tests/test_kmeans_cosine.py tests/test_kmeans_sparse_gpu.py tests/test_silhouette.py ${KM_TESTS:-} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { echo KM TESTS FAIL; grep -E "FAILED|Error|error" gpurun_out/km_tests.log | head -20; tail -30 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_km.json 2> gpurun_out/bench_km.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_km.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_km.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"] / 1e6, 1), "M rows/s", round(d["ms_per_step"], 3), "ms", r["kernel"], round(r["frac"], 3))
print({k: round(v, 3) for k, v in r["kernels_ms_per_step"].items()})
print(d.get("screen_tiers") or r.get("screen_tiers"))
PY
echo ALLDONE
# KM_AB="VAR=value ...": the bench line again with those variables set
if [ -n "${KM_AB:-}" ]; then
  env $KM_AB timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_km_ab.json 2> gpurun_out/bench_km_ab.err || { echo AB BENCH FAIL; tail -20 gpurun_out/bench_km_ab.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/bench_km_ab.json').read().strip().splitlines()[-1])
print('AB', '$KM_AB', round(d['value'] / 1e6, 1), round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['roofline']['kernels_ms_per_step'].items()})"
fi
