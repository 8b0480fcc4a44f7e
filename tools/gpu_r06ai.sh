#!/bin/bash
# KMeans two-phase re-check kernel: the carried-bounds tests, the KMeans suite, a bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmeans_gpu.py -k "incremental or carried_bounds or exact or tie or nan or dup" > gpurun_out/r06ai_pytest_inc.log 2>&1 || { tail -40 gpurun_out/r06ai_pytest_inc.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 2 > gpurun_out/r06ai_bench.json 2> gpurun_out/r06ai_bench.err || { tail -20 gpurun_out/r06ai_bench.err; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmeans_gpu.py tests/test_kmeans_model_gpu.py tests/test_kmeans_suite_init.py tests/test_dataset.py -k "not full_config" > gpurun_out/r06ai_pytest.log 2>&1 || { tail -40 gpurun_out/r06ai_pytest.log; exit 1; }
tail -1 gpurun_out/r06ai_pytest.log
timeout -k 10 420 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_kmeans_gpu.py -k "late_iteration" > gpurun_out/r06ai_pytest_full.log 2>&1 || { tail -30 gpurun_out/r06ai_pytest_full.log; exit 1; }
tail -1 gpurun_out/r06ai_pytest_full.log
