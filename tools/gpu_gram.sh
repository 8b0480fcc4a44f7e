set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gramian_gpu.py tests/test_dataset.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gram.log 2>&1 || { echo PYTEST FAIL; tail -30 gpurun_out/pytest_gram.log; exit 1; }
tail -1 gpurun_out/pytest_gram.log
timeout -k 10 300 python -u bench.py --workload gramian --cpu-seconds 0 > gpurun_out/bench_gramian.json 2> gpurun_out/bench_gramian.err || { tail gpurun_out/bench_gramian.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_gramian.json'));r=d['roofline'];print(round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],2), 'ms', r['kernel'], round(r['frac'],3))"
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gram_tiles -T -d $GRAFT_REPO_ROOT/gpurun_out/gram_fetch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-seconds 0 --workload gramian --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/gram_fetch.log 2>&1 || exit 1
python3 -c "
import csv; v=[float(r['Counter_Value']) for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/gram_fetch/run_counter_collection.csv'))]; print('FETCH_SIZE KB per dispatch', sum(v)/len(v), 'x2 GB', 2*sum(v)/len(v)*1024/1e9)"
