# Pipeline-mode experiments (DAGPU_PIPE_MODE q / d / qd): correctness of the device-batch
# tests under qd, A/B against the default, and a kernel timeline of qd.
set -o pipefail
DAGPU_PIPE_MODE=qd timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "device_batch or pipelined or mixed" --timeout 200 --timeout-method thread > gpurun_out/qd_tests.log 2>&1 || { echo "qd tests failed"; tail -5 gpurun_out/qd_tests.log; exit 1; }
echo "qd tests ok: $(tail -1 gpurun_out/qd_tests.log)"
bash tools/gpu_ab.sh "base::" "qd:DAGPU_PIPE_MODE=qd:" "qd_l3:DAGPU_PIPE_MODE=qd DAGPU_LEAF_QUEUE=3:" "qd_r2:DAGPU_PIPE_MODE=qd DAGPU_RS_QUEUE=2:" "qd_s8:DAGPU_PIPE_MODE=qd DAGPU_PIPE_SLICES=8:" "q:DAGPU_PIPE_MODE=q:" "base2::" || exit 1
bash tools/gpu_timeline.sh "qd:DAGPU_PIPE_MODE=qd" > /dev/null
