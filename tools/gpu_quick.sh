# quick GPU iteration: parity tests, bench, optional microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
if [ "$1" = "micro" ]; then timeout -k 10 120 ./tools/valu_bench > gpurun_out/valu_bench.log 2>&1; cat gpurun_out/valu_bench.log; fi
