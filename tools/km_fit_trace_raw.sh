# A KMeans fit's kernel trace, kept (gzip) as gpurun_out/kft_raw.csv.gz for a timeline
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kft
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/kft/trace -o run --output-format csv -- python3 $R/tools/probe/kmeans_fit_only.py > $R/gpurun_out/kft/trace.log 2>&1 || exit $?
f=$(find $R/gpurun_out/kft/trace -name '*kernel_trace.csv' | head -1)
gzip -c "$f" > $R/gpurun_out/kft_raw.csv.gz
m=$(find $R/gpurun_out/kft/trace -name '*memory_copy_trace.csv' | head -1)
[ -n "$m" ] && gzip -c "$m" > $R/gpurun_out/kft_copy.csv.gz
find $R/gpurun_out/kft -name '*.csv' -delete
ls -la $R/gpurun_out/kft_raw.csv.gz
