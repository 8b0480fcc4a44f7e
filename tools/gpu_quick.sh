set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kmeans_gpu.py tests/test_dataset.py tests/test_logistic_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
AB_VARIANTS=3,8 timeout -k 10 200 python -u tools/kmeans_ab.py 10000000 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -3 gpurun_out/ab.log
for w in kmeans lr_sparse; do
timeout -k 10 240 python -u bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail gpurun_out/bench_$w.err; exit 1; }
cat gpurun_out/bench_$w.json
done
bash tools/prof.sh prof_kmeans --workload kmeans --steps 3 --warmup 2 || exit 1
bash tools/prof.sh prof_lr_sparse --workload lr_sparse --steps 3 --warmup 1 || exit 1
echo ALLDONE
