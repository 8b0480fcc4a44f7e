# One workload's bench line with the in-tree library and with each
# tools/bin/libcyclone_<v>.so of $VARIANTS (built on the CPU side, e.g. with a
# probe or template define; copied over the box's scratch copy of the in-tree
# library), the in-tree library again last.  WORKLOAD (default kmeans), STEPS,
# BENCH_ARGS (more bench.py flags, e.g. --rows N).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
W=${WORKLOAD:-kmeans}
cp cycloneml_amd/libcyclone.so /tmp/libcyclone_base.so
for v in base ${VARIANTS:-} base; do
  if [ $v = base ]; then cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so; else cp tools/bin/libcyclone_$v.so cycloneml_amd/libcyclone.so; fi
  timeout -k 10 300 python -u bench.py --workload $W --steps ${STEPS:-10} --warmup 3 --cpu-seconds 0 ${BENCH_ARGS:-} 2>gpurun_out/ab_$v.err > gpurun_out/ab_$v.json || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(x,3) for k,x in {**d['roofline']['kernels_ms_per_step'], **d['roofline'].get('diag_kernels_ms_per_step', {})}.items()}, {k: round(x,3) for k,x in d.get('prep_ms',{}).items() if isinstance(x,(int,float))})"
done
cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so
