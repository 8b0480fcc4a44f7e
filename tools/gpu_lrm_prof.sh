set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_logistic_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lrm.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/pytest_lrm.log; exit 1; }
tail -2 gpurun_out/pytest_lrm.log
timeout -k 10 240 python -u bench.py --workload lr_multi --cpu-seconds 0 > gpurun_out/bench_lr_multi.json 2> gpurun_out/bench_lr_multi.err || { tail gpurun_out/bench_lr_multi.err; exit 1; }
cat gpurun_out/bench_lr_multi.json
bash tools/prof.sh prof_lr_multi --workload lr_multi --steps 3 --warmup 1 || exit 1
echo PROFDONE
