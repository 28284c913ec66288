# PMC pass over the repair bench (decode kernels): SQ issue/wait/ifetch counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_repair; mkdir -p $OUT
for P in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_WAIT_ANY SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$N -o run -- python3 bench.py --mode repair --steps 2 --warmup 1 > $OUT/$N.log 2>&1 || { echo "pmc $P failed"; tail -5 $OUT/$N.log; exit 1; }
  echo "pmc $P ok"
done
