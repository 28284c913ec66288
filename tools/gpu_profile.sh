# GPU profiling pass: VALU microbench, rocprofv3 kernel-trace stats of bench.py,
# and separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) -- one counter group per run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; mkdir -p $OUT
TAG=${1:-r01}
MODE=${2:-full}  # "counters": kernel trace and PMC passes only (no VALU microbench, no 4-vector run)
if [ "$MODE" = full ]; then
  timeout -k 10 120 "$GRAFT_REPO_ROOT/tools/valu_bench" > $OUT/valu_bench_$TAG.log 2>&1 || { echo "valu_bench failed"; cat $OUT/valu_bench_$TAG.log; exit 1; }
  cat $OUT/valu_bench_$TAG.log
fi
export DAGPU_PIPE_SLICES=1  # one launch per kernel per step: clean per-launch counters
BENCH="bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-replay --no-configs --no-check --distinct 16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$TAG -o run -- python3 $BENCH > $OUT/trace_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace_$TAG.log; exit 1; }
echo "trace ok"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_${TAG}_$N -o run -- python3 $BENCH > $OUT/pmc_${TAG}_$N.log 2>&1 || { echo "pmc $P failed"; tail -5 $OUT/pmc_${TAG}_$N.log; exit 1; }
  echo "pmc $P ok"
done
find $OUT -name "*.csv" | head -50
[ "$MODE" = full ] || exit 0
# clock check of the 4-vector encoder run (leaf kernel time after each encoder)
DAGPU_ENC_SLICED2=0 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_${TAG}s1_GRBM -o run -- python3 $BENCH > $OUT/pmc_${TAG}s1_GRBM.log 2>&1 || { echo "pmc s1 failed"; exit 1; }
echo "pmc s1 ok"
DAGPU_ENC_SLICED2=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${TAG}s1 -o run -- python3 $BENCH > $OUT/trace_${TAG}s1.log 2>&1 || { echo "trace s1 failed"; exit 1; }
echo "trace s1 ok"
