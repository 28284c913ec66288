# GPU A/B of encoder / layout variants: full -m gpu suite, then short bench runs.
# usage: bash tools/gpu_ab.sh "<label>:<env>:<bench args>" ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-replay --no-configs $args > gpurun_out/ab_$label.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_$label.log; exit $rc; fi
  python - "$label" gpurun_out/ab_$label.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], round(d["value"]), "sq/s", round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()})
PY
done
