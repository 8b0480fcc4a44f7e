set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in kmeans gramian lr_multi lr_sparse; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH $w FAIL; tail -20 gpurun_out/bench_$w.err; exit 1; }
  cat gpurun_out/bench_$w.json
done
