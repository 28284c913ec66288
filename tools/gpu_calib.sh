set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/calib -o run -- "$GRAFT_REPO_ROOT/tools/fetch_calib" > gpurun_out/prof/calib.log 2>&1 || { tail -5 gpurun_out/prof/calib.log; exit 1; }
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/calib_t -o run -- "$GRAFT_REPO_ROOT/tools/fetch_calib" >> gpurun_out/prof/calib.log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/prof/calib/run_counter_collection.csv')):
    agg[r['Kernel_Name'][:12]].append(float(r['Counter_Value']))
for k, v in agg.items():
    kib = sum(v) / len(v)
    print(k, 'FETCH_SIZE KiB', kib, 'factor to 2 GiB:', (2 << 30) / (kib * 1024))
for r in csv.DictReader(open('gpurun_out/prof/calib_t/run_kernel_stats.csv')):
    print(r['Name'][:12], 'avg us', float(r['AverageNs']) / 1e3, 'GB/s', (2 << 30) / float(r['AverageNs']))
PY
