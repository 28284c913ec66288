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
    split1024) A="--mode split --split-k 1024 --steps 3 --warmup 1";;
    repair1024) A="--mode repair --k 1024 --batch 1 --steps 2 --warmup 1";;
    split2048) A="--mode split --split-k 2048 --steps 2 --warmup 1";;
    repair2048) A="--mode repair --k 2048 --batch 1 --steps 1 --warmup 1";;
    *) echo "unknown $wl"; exit 2;;
  esac
  B="$GRAFT_REPO_ROOT/bench.py $A"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$wl/trace -o run -- python3 $B > $OUT/$wl.trace.log 2>&1 || { echo "$wl trace failed"; tail -5 $OUT/$wl.trace.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/$wl/sq -o run -- python3 $B > $OUT/$wl.sq.log 2>&1 || { echo "$wl pmc failed"; tail -5 $OUT/$wl.sq.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/$wl/grbm -o run -- python3 $B > $OUT/$wl.grbm.log 2>&1 || { echo "$wl pmc grbm failed"; exit 1; }
  echo "$wl done"
done
python3 tools/pmc_stress.py "$@" > $OUT/summary.txt
cat $OUT/summary.txt
