# Gramian on the GPU box: the Gramian tests, then the gramian bench line with
# the in-tree library and with each tools/bin/libcyclone_<v>.so of $VARIANTS
# (copied over the box's scratch copy of the in-tree library), in-tree again last.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gramian_gpu.py > gpurun_out/gram_tests.log 2>&1 || { tail -30 gpurun_out/gram_tests.log; exit 1; }
tail -1 gpurun_out/gram_tests.log
cp cycloneml_amd/libcyclone.so /tmp/libcyclone_base.so
for v in base ${VARIANTS:-} base; do
  if [ $v = base ]; then cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so; else cp tools/bin/libcyclone_$v.so cycloneml_amd/libcyclone.so; fi
  timeout -k 10 300 python -u bench.py --workload gramian --steps 10 --warmup 3 --cpu-seconds 0 2>gpurun_out/gram_$v.err > gpurun_out/gram_$v.json || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/gram_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
done
