# k = 512 Repair: kernel stats and SQ counters (decoder issue/stall picture).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/p16; mkdir -p $OUT
B="$GRAFT_REPO_ROOT/bench.py --mode repair --k 512 --batch 2 --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/grbm -o run -- python3 $B > $OUT/grbm.log 2>&1 || { echo "pmc grbm failed"; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("gpurun_out/p16/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        if "dagpu" in r["Kernel_Name"]:
            agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
s=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$s" | grep dagpu | head -12
