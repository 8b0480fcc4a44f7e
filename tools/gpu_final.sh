# Round-end validation: every GPU test + smoke (PART=tests), the bench line
# of all four workloads with CPU baselines (PART=bench), or both (default).
# The maintained tools: prof.sh (rocprofv3 stats + FETCH/WRITE passes),
# pmc_summary.py, pmc_kernel.sh / pmc_mfma.sh / pmc_pass.sh (SQ counters),
# gpu_km.sh / gpu_lr.sh / gpu_gram.sh (one workload's GPU tests + bench line),
# ab_km.sh (KMeans bench under environment switches), ab_lib.sh (a bench
# line per library variant), asm_mix.py (ISA mix), probe/ + probe_*.sh
# (kernel timing probes), screen_probe.py, rocpd_stats.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PART=${PART:-all}
if [ $PART != bench ]; then
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
fi
if [ $PART != tests ]; then
# the driver's command: every workload in one run, KMeans as the headline line
timeout -k 10 500 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_all.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_all.json").read().strip().splitlines()[-1])
for name, w in [("kmeans", d)] + list(d.get("workloads", {}).items()):
    r = w.get("roofline") or {}
    print(name, round(w["value"] / 1e6, 1), "M/s", round(w["ms_per_step"], 2), "ms",
          r.get("kernel"), round(r.get("frac", 0), 3), w.get("vs_baseline"),
          (w.get("cpu_baseline") or {}).get("value"), (w.get("fit") or {}).get("fit_ms"))
PY
fi
echo ALLDONE
