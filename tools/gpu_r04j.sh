# round 4: k = 512 decoder with the next tables of a radix-4 unit loaded one phase ahead: tests, repair A/B vs the previous build
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py" --rounds 3 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
