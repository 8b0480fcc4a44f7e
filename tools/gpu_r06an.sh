#!/bin/bash
# independent shard compactions in one launch: the KMeans suites, a bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmeans_gpu.py tests/test_kmeans_model_gpu.py tests/test_kmeans_suite_init.py tests/test_kmeans_sparse_gpu.py tests/test_kmeans_cosine.py -k "not full_config" > gpurun_out/r06an_pytest.log 2>&1 || { tail -40 gpurun_out/r06an_pytest.log; exit 1; }
tail -1 gpurun_out/r06an_pytest.log
timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r06an_bench.json 2> gpurun_out/r06an_bench.err || { tail -20 gpurun_out/r06an_bench.err; exit 1; }
python3 tools/kmsum.py gpurun_out/r06an_bench.json
