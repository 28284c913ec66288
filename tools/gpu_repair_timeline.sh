# Kernel timelines of one Repair call (host turnaround between rounds): rocprofv3
# kernel trace of bench.py --mode repair per workload, then tools/repair_timeline.py.
#   bash tools/gpu_repair_timeline.sh [workload ...]   (repair128 repair512 repair128q3 repair512q3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rtl; mkdir -p $OUT
[ $# -gt 0 ] || set -- repair128 repair512
for W in "$@"; do
  case $W in
    repair128) A="--mode repair --k 128 --batch 256";;
    repair128q3) A="--mode repair --k 128 --batch 256 --pattern q3";;
    repair512) A="--mode repair --k 512 --batch 2";;
    repair512q3) A="--mode repair --k 512 --batch 2 --pattern q3";;
    *) echo "unknown workload $W"; exit 2;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$W -o run -- python3 bench.py $A --steps 3 --warmup 1 --no-cpu > $OUT/$W.log 2>&1 || { echo "$W trace failed"; tail -20 $OUT/$W.log; exit 1; }
  CSV=$(find $OUT/$W -name "*kernel_trace.csv" | head -1)
  python3 tools/repair_timeline.py "$CSV" 3 > $OUT/${W}_timeline.txt || { echo "$W timeline failed"; exit 1; }
  head -1 $OUT/${W}_timeline.txt
done
