# Round 6: the k = 16384 split square (one part of P = 64 end to end, the
# finish step) and the split regressions.  bash tools/gpu_split16k.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_split16k.py > gpurun_out/r06_split16k.log 2>&1
rc=$?; echo "split16k rc=$rc"; tail -8 gpurun_out/r06_split16k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_parity.py > gpurun_out/r06_split16k_regress.log 2>&1
rc=$?; echo "regress rc=$rc"; tail -3 gpurun_out/r06_split16k_regress.log; [ $rc -eq 0 ] || exit $rc
