# GF(2^16) decoder A/B: GF(2^16) parity tests, then k = 256 / 512 Repair with two library builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py -k "gf16 or 256 or 512" > gpurun_out/gf16ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gf16ab_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gf16ab_tests.log | head -20; exit $rc; fi
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "default" ]; then unset DAGPU_LIB; else export DAGPU_LIB=$lib; fi
    for kb in "256:8" "512:2"; do
      kk=${kb%%:*}; bb=${kb#*:}
      timeout -k 10 200 python -u bench.py --mode repair --k $kk --batch $bb --steps 5 --warmup 1 > gpurun_out/g16ab_${label}_${kk}_$rep.log 2>&1 || { echo "$label k=$kk failed"; tail -5 gpurun_out/g16ab_${label}_${kk}_$rep.log; exit 1; }
      echo "$label k$kk $(tail -1 gpurun_out/g16ab_${label}_${kk}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
    done
  done
done
unset DAGPU_LIB
