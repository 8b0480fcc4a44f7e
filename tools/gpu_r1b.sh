set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for w in kmeans gramian lr_multi lr_sparse; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  cat gpurun_out/bench_$w.json
done
