# Full GPU parity suite, then the headline bench and the repair benches (k = 128 / 256 / 512).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-replay --no-e2e --no-configs > gpurun_out/hl.log 2>&1 || { echo "headline failed"; tail -5 gpurun_out/hl.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/hl.log') if l.startswith('{')][-1])
print('headline', round(d['value']), round(d['ms_per_step'],3), d.get('headline_bit_exact'))"
for kb in "128 256" "256 8" "512 2"; do
  set -- $kb
  timeout -k 10 200 python -u bench.py --mode repair --k $1 --batch $2 --steps 5 --warmup 1 > gpurun_out/rep_$1.log 2>&1 || { echo "repair bench k=$1 failed"; tail -5 gpurun_out/rep_$1.log; exit 1; }
  echo "repair k$1 $(tail -1 gpurun_out/rep_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
done
