# Cosine KMeans GPU tests, then (unless they crashed) the round-2 profiles
# of the workloads named in WL.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_cosine.py -x -v --timeout 300 --timeout-method thread > gpurun_out/cos.log 2>&1
rc=$?
tail -5 gpurun_out/cos.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$WL" ] && WL="$WL" bash tools/gpu_prof_r02.sh
echo ALLDONE
