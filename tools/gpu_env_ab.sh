# A/B of runtime settings on the headline step: bash tools/gpu_env_ab.sh [--tests] label=VAR=v,VAR=v ...
# ("label=" alone = defaults).  Interleaved, two rounds; optional parity subset first.
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "--tests" ]; then
  shift
  timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_checks.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pipelined" > gpurun_out/envab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/envab_tests.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/envab_tests.log | head -20; exit $rc; fi
fi
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; vars=${spec#*=}
    envs=$(echo "$vars" | tr ',' ' ')
    timeout -k 10 200 env $envs python -u bench.py --steps 20 --warmup 3 --no-cpu --no-replay --no-e2e --no-configs > gpurun_out/envab_${label}_$rep.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/envab_${label}_$rep.log; exit $rc; fi
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/envab_${label}_$rep.log') if l.startswith('{')][-1])
print('$label', round(d['value']), round(d['ms_per_step'],3), d.get('headline_bit_exact'))"
  done
done
