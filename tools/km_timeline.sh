# One KMeans iteration's kernel timeline under rocprofv3 --kernel-trace
# (tools/trace_timeline.py), written to gpurun_out/km_timeline.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/kmt
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kmt/trace -o run --output-format csv -- python3 $R/bench.py --workload kmeans --steps 5 --warmup 3 --cpu-seconds 0 > $R/gpurun_out/kmt/trace.log 2>&1 || exit $?
f=$(find $R/gpurun_out/kmt/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_timeline.py "$f" "${MARK:-k_screen32<8, 4, 1, false>}" ${BACK:-2} > $R/gpurun_out/km_timeline.txt
find $R/gpurun_out/kmt -name '*.csv' -delete
tail -3 $R/gpurun_out/km_timeline.txt
