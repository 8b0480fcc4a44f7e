set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kmeans_gpu.py tests/test_kmeans_model_gpu.py tests/test_kmeans_sparse_gpu.py tests/test_dataset.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error|assert" gpurun_out/pytest_km.log | head -20; tail -30 gpurun_out/pytest_km.log; exit 1; }
tail -2 gpurun_out/pytest_km.log
timeout -k 10 300 python -u bench.py --workload kmeans --cpu-seconds 0 > gpurun_out/bench_kmeans.json 2> gpurun_out/bench_kmeans.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_kmeans.err; exit 1; }
cat gpurun_out/bench_kmeans.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/km_prof -o km -- python3 -u bench.py --workload kmeans --cpu-seconds 0 --steps 5 --warmup 2 > gpurun_out/km_prof.log 2>&1 || { echo PROF FAIL; tail -20 gpurun_out/km_prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/km_prof/km_results.db 8
if [ -n "$PMC" ]; then timeout -k 10 400 bash tools/pmc_mfma.sh km2 k_screen32 --workload kmeans > gpurun_out/pmc_km2.txt 2>&1 && cat gpurun_out/pmc_km2.txt; fi
