# Round profiles in one GPU call: rocprofv3 stats + FETCH/WRITE passes per
# workload (tools/prof.sh), summarised on the box into
# gpurun_out/<tag>_<workload>/summary_{pmc.json,kernel_stats.csv}.
# usage: TAG=r05 WLS="kmeans gramian pca lr_multi" bash tools/prof_all.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
declare -A ROWS=([kmeans]=10000000 [gramian]=30000000 [pca]=30000000 [lr_multi]=50000000 [lr_sparse]=200000000)
for w in ${WLS:-kmeans gramian pca lr_multi}; do
  SUMMARY=${ROWS[$w]}:${ITERS:-8} bash tools/prof.sh ${TAG:-r05}_$w --workload $w --steps ${STEPS:-5} --warmup 3 || { echo PROF FAIL $w; tail -5 gpurun_out/${TAG:-r05}_$w/*.log; exit 1; }
  echo "$w profiled"
done
echo PROFDONE
