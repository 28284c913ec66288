# GF(2^16) stress workloads (configs[4] widths): kernel-trace stats and SQ/GRBM counters per
# launch of the GF(2^16) kernels, one rocprofv3 run per pass (counters never combined with
# trace domains).  Summary: gpurun_out/p16/summary.txt
#   bash tools/gpu_pmc_gf16.sh [workload ...]   (repair512 repair512q3 split512 repair256 repair128)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/p16; mkdir -p $OUT
[ $# -gt 0 ] || set -- repair512 repair512q3 split512
for wl in "$@"; do
  case $wl in
    repair512) A="--mode repair --k 512 --batch 2 --steps 3 --warmup 1";;
    repair512q3) A="--mode repair --k 512 --batch 2 --steps 3 --warmup 1 --pattern q3";;
    repair256) A="--mode repair --k 256 --batch 8 --steps 3 --warmup 1";;
    split512) A="--mode split --split-k 512 --steps 3 --warmup 1";;
    repair128) A="--mode repair --k 128 --batch 256 --steps 3 --warmup 1";;
    *) echo "unknown $wl"; exit 2;;
  esac
  B="$GRAFT_REPO_ROOT/bench.py $A"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$wl/trace -o run -- python3 $B > $OUT/$wl.trace.log 2>&1 || { echo "$wl trace failed"; tail -5 $OUT/$wl.trace.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/$wl/sq -o run -- python3 $B > $OUT/$wl.sq.log 2>&1 || { echo "$wl pmc failed"; tail -5 $OUT/$wl.sq.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/$wl/grbm -o run -- python3 $B > $OUT/$wl.grbm.log 2>&1 || { echo "$wl pmc grbm failed"; exit 1; }
  echo "$wl done"
done
python3 - "$@" > $OUT/summary.txt <<'PY'
import csv, glob, collections, re, sys
def kname(n):
    return n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
for wl in sys.argv[1:]:
    print(f"== {wl}")
    s = glob.glob(f"gpurun_out/p16/{wl}/trace/**/*kernel_stats.csv", recursive=True)
    if s:
        rows = list(csv.DictReader(open(s[0])))
        for r in rows[:14]:
            print(f"  stats {kname(r['Name'])[:70]:70s} calls {r['Calls']:>5s} avg_ms {float(r['AverageNs'])/1e6:.4f} pct {float(r['Percentage']):.1f}")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(f"gpurun_out/p16/{wl}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            n = kname(r["Kernel_Name"])
            if "leo16" in n or "errloc" in n or "decode128" in n:
                agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, d in sorted(agg.items()):
        a = {c: sum(v) / len(v) for c, v in d.items()}
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
        valu = a.get("SQ_INSTS_VALU", 0)
        waves = a.get("SQ_WAVES", 0)
        out = {c: round(v) for c, v in a.items()}
        if cyc and valu:
            out["valu_per_clk_per_cu"] = round(valu / cyc / 256, 3)
        if waves:
            out["valu_per_wave"] = round(valu / waves)
        if a.get("SQ_WAVE_CYCLES"):
            out["wait_inst_frac"] = round(a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"], 3)
            out["wait_any_frac"] = round(a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"], 3)
        print(f"  pmc {n[:80]} {out}")
PY
cat $OUT/summary.txt
