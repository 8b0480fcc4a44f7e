set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for w in kmeans gramian lr_multi lr_sparse; do
  bash tools/prof.sh prof_$w --workload $w --steps 3 --warmup 1 || { echo PROF $w FAIL; tail -20 gpurun_out/prof_$w/*.log; exit 1; }
  echo done $w
done
