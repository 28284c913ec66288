# Repair reverse fill: parity (fill tests incl. the reverse patterns + the repair
# suites), then the repair bench with the random sub-grid (configs[3]) and the
# Q3-only pattern, shortcut on/off, and the previous build (DAGPU_LIB) for A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_repair_fill.py > gpurun_out/rfill_tests.log 2>&1
rc=$?; echo "fill tests rc=$rc"; tail -6 gpurun_out/rfill_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/rfill_tests.log | head -20; exit $rc; fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_gf16.py -k "repair or decode or byz or codec or erasure" > gpurun_out/rfill_tests2.log 2>&1
rc=$?; echo "repair suites rc=$rc"; tail -3 gpurun_out/rfill_tests2.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/rfill_tests2.log | head -20; exit $rc; fi
run() {  # label env... -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --mode repair --steps 5 --warmup 1 ${BARGS} > gpurun_out/rfill_${label}.log 2>&1 || { echo "$label failed"; tail -5 gpurun_out/rfill_${label}.log; exit 1; }
  echo "$label $(tail -1 gpurun_out/rfill_${label}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
}
for kb in "128 256" "256 8" "512 2"; do
  set -- $kb
  for pat in q3 subgrid; do
    BARGS="--k $1 --batch $2 --pattern $pat"
    run "k$1_${pat}_new" DAGPU_REPAIR_FILL=1
    run "k$1_${pat}_prev" DAGPU_REPAIR_FILL=1 DAGPU_LIB=celestia-app_amd/libdagpu_prev.so
    run "k$1_${pat}_nofill" DAGPU_REPAIR_FILL=0
  done
done
