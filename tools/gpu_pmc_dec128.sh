# k = 128 Repair: SQ counters of the bit-sliced decoder (issue, stalls, LDS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pd128; mkdir -p $OUT
B="$GRAFT_REPO_ROOT/bench.py --mode repair --steps 2 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/grbm -o run -- python3 $B > $OUT/grbm.log 2>&1 || { echo "pmc2 failed"; tail -5 $OUT/grbm.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("gpurun_out/pd128/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"]
        if "decode128_sliced" in n or "encode_sliced2_kernel<true>" in n or "nmt_leaf" in n:
            agg[n.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(max(v)) for c, v in d.items()})
PY
