set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_logistic_gpu.py tests/test_lr_fit.py tests/test_dataset.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lrm.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error|error" gpurun_out/pytest_lrm.log | head; tail -30 gpurun_out/pytest_lrm.log; exit 1; }
tail -2 gpurun_out/pytest_lrm.log
timeout -k 10 300 python -u bench.py --workload lr_multi --cpu-seconds 0 > gpurun_out/bench_lr_multi.json 2> gpurun_out/bench_lr_multi.err || { tail gpurun_out/bench_lr_multi.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_lr_multi.json'));r=d['roofline'];print(round(d['value']/1e6,1), 'M rows/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['frac'],3), {k: round(v,2) for k,v in r['kernels_ms_per_step'].items()})"
