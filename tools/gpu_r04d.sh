# round 4: GF(2^16) k = 512 decoder (two-group perms, paired-lane loads): tests, then A/B vs the previous build
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py" --rounds 2 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so
