# GF(2^16) encoder occupancy A/B: parity (gf16 + fill tests), then the k = 512 / 256
# Q3 repair (reverse-fill encodes), the subgrid repair and the split stress square
# with the in-tree build and DAGPU_LIB=<prev build>.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py > gpurun_out/g16e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g16e_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/g16e_tests.log | head -20; exit $rc; fi
for rep in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export DAGPU_LIB=celestia-app_amd/libdagpu_prev.so; else unset DAGPU_LIB; fi
    for spec in "512 2 q3" "256 8 q3" "512 2 subgrid"; do
      set -- $spec
      timeout -k 10 200 python -u bench.py --mode repair --k $1 --batch $2 --pattern $3 --steps 4 --warmup 1 > gpurun_out/g16e_${lib}_$1_$3_$rep.log 2>&1 || { echo "$lib $spec failed"; tail -5 gpurun_out/g16e_${lib}_$1_$3_$rep.log; exit 1; }
      echo "$lib k$1 $3 $(tail -1 gpurun_out/g16e_${lib}_$1_$3_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
    done
    timeout -k 10 200 python -u bench.py --mode split --steps 3 --warmup 1 > gpurun_out/g16e_${lib}_split_$rep.log 2>&1 || { echo "$lib split failed"; tail -5 gpurun_out/g16e_${lib}_split_$rep.log; exit 1; }
    echo "$lib split $(tail -1 gpurun_out/g16e_${lib}_split_$rep.log | cut -c1-300)"
  done
done
unset DAGPU_LIB
