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
  # the summaries come back (gpurun returns gpurun_out/ only, <= 64 MiB): the
  # raw per-dispatch traces stay behind
  mkdir -p gpurun_out/profiles && cp profiles/r02_${w}_kernel_stats.csv profiles/r02_${w}_pmc.json gpurun_out/profiles/
  rm -f gpurun_out/prof_$w/*/run_kernel_trace.csv gpurun_out/prof_$w/*/run_counter_collection.csv
  echo done $w
done
