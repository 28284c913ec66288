set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rtl; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/k128 -o run -- python3 bench.py --mode repair --steps 3 --warmup 1 > $OUT/k128.log 2>&1 || { echo "trace failed"; tail -5 $OUT/k128.log; exit 1; }
f=$(find $OUT/k128 -name "*kernel_trace.csv" | head -1)
python3 tools/repair_timeline.py "$f" 3 > $OUT/k128.txt && cat $OUT/k128.txt
