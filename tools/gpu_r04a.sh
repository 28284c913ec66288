set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_trees.py > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_sub.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/single_square.py 2 > gpurun_out/single_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep round gpurun_out/single_ab.log
exit $rc
