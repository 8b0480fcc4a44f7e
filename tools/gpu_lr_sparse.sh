# Logistic GPU tests, then the lr_sparse bench line (200M-row config 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_logistic_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { echo LR TESTS FAIL; grep -E "FAILED|Error" gpurun_out/lr_tests.log | head; tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
timeout -k 10 600 python -u bench.py --workload lr_sparse --steps 5 --warmup 2 ${CPU:+--cpu-seconds $CPU} > gpurun_out/bench_lr_sparse.json 2> gpurun_out/bench_lr_sparse.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_lr_sparse.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_lr_sparse.json'));print(round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', d['roofline']['kernels_ms_per_step'], round(d['roofline']['frac'],3))"
