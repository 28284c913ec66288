# Kernel timeline of the pipelined headline step: rocprofv3 kernel trace of a
# short bench run per configuration (env given as arguments), summarised by
# tools/timeline.py (per-kernel start/end within the last timed step).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tl; mkdir -p $OUT
BENCH="bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-replay --no-configs --distinct 16"
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$label -o run -- python3 $BENCH > $OUT/$label.log 2>&1 || { echo "$label failed"; tail -20 $OUT/$label.log; exit 1; }
  f=$(find $OUT/$label -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py "$f" > $OUT/$label.txt || exit 1
  echo "== $label"; cat $OUT/$label.txt
done
