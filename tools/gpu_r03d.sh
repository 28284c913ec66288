# full -m gpu suite, then the default bench exactly as the driver runs it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_full.log
