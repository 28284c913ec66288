set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
BENCH="bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --batch 64 --distinct 8"
for v in 0 1; do
DAGPU_BS=$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_IFETCH SQ_INSTS_SALU --output-format csv -d gpurun_out/prof/bs$v -o run -- python3 $BENCH > gpurun_out/prof/bs$v.log 2>&1 || { tail -5 gpurun_out/prof/bs$v.log; exit 1; }
python3 - <<PY
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open('gpurun_out/prof/bs$v/run_counter_collection.csv')):
    if 'encode' in r['Kernel_Name']:
        agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items(): print('BS=$v', k, {c: round(sum(v)/len(v)) for c, v in d.items()})
PY
done
