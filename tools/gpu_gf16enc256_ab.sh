# GF(2^16) M = 256 encoder occupancy A/B (waves_per_eu 2 vs 3): k = 256 Q3 repair and split square, in-tree build vs DAGPU_LIB prev.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gf16.py > gpurun_out/g256_tests.log 2>&1 || { tail -5 gpurun_out/g256_tests.log; exit 1; }
tail -1 gpurun_out/g256_tests.log
for rep in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export DAGPU_LIB=celestia-app_amd/libdagpu_prev.so; else unset DAGPU_LIB; fi
    timeout -k 10 200 python -u bench.py --mode repair --k 256 --batch 8 --pattern q3 --steps 5 --warmup 1 > gpurun_out/g256_${lib}_q3_$rep.log 2>&1 || exit 1
    echo "$lib k256 q3 $(tail -1 gpurun_out/g256_${lib}_q3_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3), d["bit_exact"])')"
    timeout -k 10 200 python -u bench.py --mode split --split-k 256 --steps 5 --warmup 1 > gpurun_out/g256_${lib}_split_$rep.log 2>&1 || exit 1
    echo "$lib split256 $(tail -1 gpurun_out/g256_${lib}_split_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3))')"
  done
done
