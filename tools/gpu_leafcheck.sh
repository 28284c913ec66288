set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_sub.log 2>&1 || { tail -20 gpurun_out/gpu_sub.log; exit 1; }
tail -1 gpurun_out/gpu_sub.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['kernel_ms_per_step'])"
BENCH="bench.py --steps 5 --warmup 1 --no-cpu --batch 64 --distinct 8"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/leaf_fetch -o run -- python3 $BENCH > gpurun_out/prof/leaf_fetch.log 2>&1 || { tail -5 gpurun_out/prof/leaf_fetch.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for p in glob.glob('gpurun_out/prof/leaf_fetch/run_counter_collection.csv'):
    for r in csv.DictReader(open(p)):
        if 'dagpu' in r['Kernel_Name']:
            agg[r['Kernel_Name'][:50]].append(float(r['Counter_Value']))
for k, v in agg.items(): print(k, 'FETCH_SIZE KiB avg', sum(v)/len(v))
PY
