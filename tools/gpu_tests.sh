# run a subset of GPU tests: bash tools/gpu_tests.sh <pytest args...>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread "$@" > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_sub.log
exit $rc
