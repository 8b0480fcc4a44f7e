#!/bin/bash
# KMeans: carried bounds for the candidate rows too -- tests, probe, bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmeans_gpu.py -k "carried_bounds or one_limb_refinement or three_limb_candidate or lloyd" > gpurun_out/r06c_pytest.log 2>&1 || { tail -30 gpurun_out/r06c_pytest.log; exit 1; }
timeout -k 10 300 python -u tools/probe/kmeans_bounds_probe.py 20 > gpurun_out/r06c_bounds_probe.jsonl 2> gpurun_out/r06c_probe.err || exit 1
timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 2 > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || exit 1
timeout -k 10 420 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_kmeans_gpu.py -k "late_iteration or third_iteration" > gpurun_out/r06c_pytest_full.log 2>&1
