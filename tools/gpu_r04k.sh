# round 4: GF(2^16) fill encoders read the out-half presence before the transform (one ballot) instead of per element in the store loop: tests, A/B
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_gf16.py" --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1 --pattern q3" new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 1 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
