# Sparse-LR tiles-pass probes: the lr_sparse bench line with libcyclone built
# with CYC_TILES_PROBE bits (tools/bin/libcyclone_t<bits>.so, copied over the
# box's in-tree library; the box's tree is a scratch copy).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp cycloneml_amd/libcyclone.so /tmp/libcyclone_base.so
for v in ${PROBES:-base t1 t2 t3}; do
  if [ $v = base ]; then cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so; else cp tools/bin/libcyclone_$v.so cycloneml_amd/libcyclone.so; fi
  timeout -k 10 300 python -u bench.py --workload lr_sparse --steps 10 --warmup 3 --cpu-seconds 0 2>gpurun_out/probe_$v.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],2), {k: round(x,2) for k,x in d['roofline']['kernels_ms_per_step'].items()})" || exit 1
done
cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so
