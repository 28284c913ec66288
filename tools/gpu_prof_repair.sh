# Repair (C4) bench + kernel-trace stats of the same command.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_repair; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode repair > $OUT/bench_repair.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench_repair.log; exit 1; }
tail -c 1500 $OUT/bench_repair.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --mode repair --steps 3 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
echo trace ok
