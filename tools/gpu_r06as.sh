#!/bin/bash
# the re-check forms test, then the closing run (every GPU test, smoke, the bench line of every workload)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_kmeans_gpu.py -k "recheck_forms" > gpurun_out/r06as_pytest_forms.log 2>&1 || { tail -40 gpurun_out/r06as_pytest_forms.log; exit 1; }
tail -1 gpurun_out/r06as_pytest_forms.log
bash tools/gpu_final.sh
