set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_checks.py tests/test_gpu_c_client.py > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_sub.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_rehearse_multi.sh 2 4 8 > gpurun_out/rehearse_multi.log 2>&1
rc=$?; echo "rehearse rc=$rc"; cat gpurun_out/rehearse_multi.log
exit $rc
