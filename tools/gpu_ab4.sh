# A/B of library builds: headline step and k=128 repair, interleaved, after a
# parity subset (codec, repair, sliced paths) on the default build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair_byz.py tests/test_gpu_bench_checks.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not rccl and not rehearsal and not corruption" > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/ab_tests.log | head -20; exit $rc; fi
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "default" ]; then unset DAGPU_LIB; else export DAGPU_LIB=$lib; fi
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-replay --no-e2e --no-configs > gpurun_out/ab_${label}_$rep.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_${label}_$rep.log; exit $rc; fi
    timeout -k 10 200 python -u bench.py --mode repair --steps 5 --warmup 1 > gpurun_out/abr_${label}_$rep.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$label repair rc=$rc"; tail -5 gpurun_out/abr_${label}_$rep.log; exit $rc; fi
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_${label}_$rep.log') if l.startswith('{')][-1])
r=json.loads([l for l in open('gpurun_out/abr_${label}_$rep.log') if l.startswith('{')][-1])
k=d['kernel_ms_per_step']
print('$label', round(d['value']), round(d['ms_per_step'],3), {x: round(v,3) for x,v in k.items()}, d.get('headline_bit_exact'), 'repair', round(r['value']), round(r['ms_per_step'],3))"
  done
done
unset DAGPU_LIB
