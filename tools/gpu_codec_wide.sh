set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide.py -k "codec_beyond or too_few or encode_matches or decode_matches" > gpurun_out/r06_codec_wide.log 2>&1
rc=$?; echo "codec tests rc=$rc"; tail -5 gpurun_out/r06_codec_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_gf16.py tests/test_gpu_split.py > gpurun_out/r06_codec_regress.log 2>&1
rc=$?; echo "regress rc=$rc"; tail -3 gpurun_out/r06_codec_regress.log; [ $rc -eq 0 ] || exit $rc
