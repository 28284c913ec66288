# Round-3 final pass: GPU suite, the driver-shaped default bench, and the profile
# pass (kernel stats + PMC groups) of the headline step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_full.log; exit 1; }
echo "bench ok"
bash tools/gpu_profile_r03.sh ${1:-r03b}
