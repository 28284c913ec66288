# round 4: GF(2^16) encoder with the last IFFT / first FFT layers merged (no scratch): tests, A/B vs the previous build
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py" --rounds 2 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 1 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
