# Round-3 profile pass of the headline step (k=128, 256 squares): rocprofv3
# kernel-trace stats, then one PMC group per run (FETCH_SIZE / WRITE_SIZE / SQ / GRBM).
# DAGPU_PIPE_SLICES=1: one launch per kernel per step, so per-launch counters and
# the bench's own per-kernel HIP-event times describe the same launches.
set -o pipefail
TAG=${1:-r03}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; mkdir -p $OUT
export DAGPU_PIPE_SLICES=1
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-replay --no-configs --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$TAG -o run -- python3 $BENCH > $OUT/trace_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace_$TAG.log; exit 1; }
grep '^{' $OUT/trace_$TAG.log | tail -1 | cut -c1-300
echo "trace ok"
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_${TAG}_$N -o run -- python3 $BENCH > $OUT/pmc_${TAG}_$N.log 2>&1 || { echo "pmc $P failed"; tail -5 $OUT/pmc_${TAG}_$N.log; exit 1; }
  echo "pmc $P ok"
done
