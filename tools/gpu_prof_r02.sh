# Round-2 profiles: per workload a kernel trace + stats pass and separate
# FETCH_SIZE / WRITE_SIZE passes (tools/prof.sh), summarised into
# profiles/r02_<workload>_{kernel_stats.csv,pmc.json}; then the MFMA-busy pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out profiles
for w in ${WL:-kmeans gramian}; do
  bash tools/prof.sh prof_$w --workload $w --steps 3 --warmup 1 || { echo PROF $w FAIL; tail -20 gpurun_out/prof_$w/*.log; exit 1; }
  rows=$(python -c "import bench; print(bench.DEFAULT_ROWS['$w'])")
  python tools/pmc_summary.py gpurun_out/prof_$w profiles/r02_$w $rows 4 > gpurun_out/prof_$w/summary.txt || exit 1
  echo done $w
done
