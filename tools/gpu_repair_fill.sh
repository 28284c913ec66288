# Repair fill route / deferral: parity (new tests + the existing repair suites), then
# the configs[3] repair bench and k = 256 / 512 with the shortcut on and off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_repair_fill.py > gpurun_out/fill_tests.log 2>&1
rc=$?; echo "fill tests rc=$rc"; tail -12 gpurun_out/fill_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/fill_tests.log | head -20; exit $rc; fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_gf16.py -k "repair or decode or byz or codec or erasure" > gpurun_out/fill_tests2.log 2>&1
rc=$?; echo "repair suites rc=$rc"; tail -3 gpurun_out/fill_tests2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/fill_tests2.log | head -20; exit $rc; fi
for rep in 1 2; do
  for f in 1 0; do
    DAGPU_REPAIR_FILL=$f timeout -k 10 200 python -u bench.py --mode repair --steps 5 --warmup 1 > gpurun_out/fill_r128_${f}_$rep.log 2>&1 || { echo "repair bench failed"; tail -5 gpurun_out/fill_r128_${f}_$rep.log; exit 1; }
    echo "k128 fill=$f $(tail -1 gpurun_out/fill_r128_${f}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3), d["bit_exact"])')"
  done
done
for kb in "256 8" "512 2"; do
  set -- $kb
  for f in 1 0; do
    DAGPU_REPAIR_FILL=$f timeout -k 10 200 python -u bench.py --mode repair --k $1 --batch $2 --steps 3 --warmup 1 > gpurun_out/fill_r$1_$f.log 2>&1 || { echo "repair bench k=$1 failed"; tail -5 gpurun_out/fill_r$1_$f.log; exit 1; }
    echo "k$1 fill=$f $(tail -1 gpurun_out/fill_r$1_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
  done
done
