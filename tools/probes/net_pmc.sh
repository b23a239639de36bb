set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/netpmc
timeout -k 10 300 python3 -u bench.py --config C4 --steps 4 --warmup 1 --no-secondary --no-cpu-baseline --batch 1024 > gpurun_out/netpmc/bench.log 2>&1 || exit 1
tail -1 gpurun_out/netpmc/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']['module_net_kernel']; print('value', d['value'], 'net ms', k['avg_ms'], 'frac', k['frac'])"
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/netpmc/p -o run -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --batch 1024 > gpurun_out/netpmc/p.log 2>&1 || exit 1
python3 - <<'PY'
import csv,collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open('gpurun_out/netpmc/p/run_counter_collection.csv')):
    if 'net_kernel' in r['Kernel_Name']:
        agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k,d in agg.items(): print(k, {c: f"{sum(v)/len(v):.3g}" for c,v in d.items()})
PY
