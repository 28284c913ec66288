# GF(2^16) decode/repair parity with the folded error locators, k=512/256 repair
# A/B (fold vs 65536-point form), then the single-square latency block of bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gf16.py tests/test_gpu_repair_byz.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gf16_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gf16_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gf16_tests.log | head -20; exit $rc; fi
for rep in 1 2; do
for spec in "fold512::--k 512 --batch 2" "full512:DAGPU_ERRLOC_FULL=1:--k 512 --batch 2" "fold256::--k 256 --batch 8" "full256:DAGPU_ERRLOC_FULL=1:--k 256 --batch 8"; do
  label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python -u bench.py --mode repair --steps 5 --warmup 1 $args > gpurun_out/rep_$label.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/rep_$label.log; exit $rc; fi
  echo "$label $(tail -1 gpurun_out/rep_$label.log | cut -c1-150)"
done
done
timeout -k 10 300 python -u -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'celestia-app_amd')
import bench
from celestia_da import da
r = bench.bench_single(da.Context(0))
for k, v in r.items():
    print(k, {m: (round(v[m]['p50_ms'], 3), round(v[m]['p99_ms'], 3)) for m in ('roots_only', 'with_eds', 'with_eds_pageable')})
json.dump(r, open('gpurun_out/single.json', 'w'))
" > gpurun_out/single.log 2>&1; echo "single rc=$?"; tail -3 gpurun_out/single.log
