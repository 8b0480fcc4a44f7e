# The bench line's dominant-kernel time against rocprofv3's trace of the same
# command: gpurun_out/${TAG}_agree.txt (the timed launches picked by order)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kag
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kag/t -o run --output-format csv -- python3 $R/bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/kag/bench.json 2> $R/gpurun_out/kag/bench.err || exit $?
f=$(find $R/gpurun_out/kag/t -name '*kernel_trace.csv' | head -1)
st=$(find $R/gpurun_out/kag/t -name '*kernel_stats.csv' | head -1)
cp "$st" $R/gpurun_out/${TAG}_kmeans_trace_stats.csv
python3 $R/tools/agree_summary.py "$f" $R/gpurun_out/kag/bench.json k_recheck 4 20 > $R/gpurun_out/${TAG}_agree.txt
find $R/gpurun_out/kag -name '*.csv' -delete
cat $R/gpurun_out/${TAG}_agree.txt
