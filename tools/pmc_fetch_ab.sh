# FETCH_SIZE (one --pmc pass each) of one kernel under the in-tree library
# and each tools/bin/libcyclone_<v>.so of $VARIANTS; WORKLOAD, KRX (kernel
# regex), BENCH_ARGS.  Prints the mean raw FETCH_SIZE (KB) per dispatch.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
cp cycloneml_amd/libcyclone.so /tmp/libcyclone_base.so
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so; else cp tools/bin/libcyclone_$v.so cycloneml_amd/libcyclone.so; fi
  rm -rf /tmp/pmcab_$v
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" -d /tmp/pmcab_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $WORKLOAD --steps 2 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > /tmp/pmcab_$v.log 2>&1) || { tail -5 /tmp/pmcab_$v.log; cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
vals = [float(r["Counter_Value"]) for f in glob.glob(f"/tmp/pmcab_{v}/**/run_counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
print(v, "FETCH_SIZE KB raw per dispatch", sum(vals) / max(1, len(vals)), "n", len(vals))
PY
done
cp /tmp/libcyclone_base.so cycloneml_amd/libcyclone.so
