# Repair A/B: full -m gpu suite, then configs[3] repair bench runs per env spec.
# usage: bash tools/gpu_repair_ab.sh "<label>:<env>:<bench args>" ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python -u bench.py --mode repair --steps 5 --warmup 1 $args > gpurun_out/rep_$label.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/rep_$label.log; exit $rc; fi
  echo "$label $(tail -1 gpurun_out/rep_$label.log)"
done
