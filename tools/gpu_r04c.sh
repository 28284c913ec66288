# round 4: started Repairs (dagpu_repair_start / join) -- tests, then one batch
# vs 2 started slices (k = 128 and 512)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_repair_async.py tests/test_gpu_repair_fill.py > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_sub.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh --rounds 2 repair128 one= "slices2=args:--repair-slices 2" && \
bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 512 --batch 4 --steps 4 --warmup 1" one= "slices2=args:--repair-slices 2"
