set -o pipefail
cd $GRAFT_REPO_ROOT
for w in kmeans gramian lr_multi lr_sparse; do
  bash tools/prof.sh prof_$w --workload $w --steps 3 --warmup 1 || { echo PROF $w FAIL; tail -20 gpurun_out/prof_$w/*.log; exit 1; }
  echo done $w
done
