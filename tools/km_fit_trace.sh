# A KMeans fit's kernel trace, summarised per iteration into gpurun_out/km_fit_trace.txt
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kft
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kft/trace -o run --output-format csv -- python3 $R/tools/probe/kmeans_fit_only.py > $R/gpurun_out/kft/trace.log 2>&1 || exit $?
f=$(find $R/gpurun_out/kft/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/fit_trace_summary.py "$f" > $R/gpurun_out/km_fit_trace.txt
find $R/gpurun_out/kft -name '*.csv' -delete
head -60 $R/gpurun_out/km_fit_trace.txt
