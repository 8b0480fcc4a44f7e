# KMeans bench line under each environment setting of $SETTINGS (";"-separated,
# e.g. "A=1;A=2 B=0"; "-" = none), one bench process each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
IFS=';' read -ra SET <<< "${SETTINGS:--}"
i=0
for e in "${SET[@]}"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python -u bench.py --workload kmeans --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -5 gpurun_out/ab_$i.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/ab_$i.json').read().strip().splitlines()[-1])
print('[$e]', round(d['value'] / 1e6, 1), round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['roofline']['kernels_ms_per_step'].items()})"
done
