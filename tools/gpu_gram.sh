# Gramian on the GPU box: the Gramian tests and the gramian bench line under
# each kernel of $KERNELS (CYC_GRAMIAN_KERNEL; "-" = the default).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in ${KERNELS:--}; do
  e=""; [ "$k" != "-" ] && e="CYC_GRAMIAN_KERNEL=$k"
  env $e timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gramian_gpu.py > gpurun_out/gram_tests_$k.log 2>&1 || { echo "TESTS FAIL $k"; tail -30 gpurun_out/gram_tests_$k.log; exit 1; }
  echo "$k $(tail -1 gpurun_out/gram_tests_$k.log)"
done
for k in ${KERNELS:--}; do
  e=""; [ "$k" != "-" ] && e="CYC_GRAMIAN_KERNEL=$k"
  env $e timeout -k 10 300 python -u bench.py --workload gramian --steps 10 --warmup 3 --cpu-seconds 0 2>gpurun_out/gram_$k.err > gpurun_out/gram_$k.json || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/gram_$k.json').read().strip().splitlines()[-1]); print('$k', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
done
