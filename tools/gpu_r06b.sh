#!/bin/bash
# round 6 batch: new GPU tests, the carried-bounds probe, the MALL residency
# probe (tools/probe/tiles_mall_probe.py), a KMeans bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_abi_threads.py tests/test_logistic_gpu.py::test_tiles_auto_demotes_to_wide tests/test_gramian_gpu.py::test_covariance_entrywise_mixed_scales tests/test_gramian_gpu.py::test_covariance_form_choice > gpurun_out/r06b_pytest.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python -u tools/probe/kmeans_bounds_probe.py 20 > gpurun_out/r06b_bounds_probe.jsonl 2> gpurun_out/r06b_probe.err || exit 1
CYC_LIB_DIR=tools/bin/mall timeout -k 10 300 python -u tools/probe/tiles_mall_probe.py 229376:2:20 16777216:4:1 > gpurun_out/r06b_mall_probe.jsonl 2> gpurun_out/r06b_mall.err || exit 1
timeout -k 10 200 python -u tools/probe/tiles_mall_probe.py 16777216:1:1 >> gpurun_out/r06b_mall_probe.jsonl 2>> gpurun_out/r06b_mall.err || exit 1
timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 2 > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err
