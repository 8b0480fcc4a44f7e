# rocprofv3 kernel stats of a short KMeans bench: gpurun_out/${TAG}_stats.csv
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kst
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kst/t -o run --output-format csv -- python3 $R/bench.py --workload kmeans --steps 10 --warmup 3 --cpu-seconds 0 > $R/gpurun_out/kst/log 2>&1 || exit $?
f=$(find $R/gpurun_out/kst/t -name '*kernel_stats.csv' | head -1)
cp "$f" $R/gpurun_out/${TAG}_stats.csv
find $R/gpurun_out/kst -name '*.csv' -delete
grep -E "stats_pairs|require_norms|k_recheck|bounds_filter" $R/gpurun_out/${TAG}_stats.csv | cut -c1-160
