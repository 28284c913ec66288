# round 4: k = 128 sliced fill encoder reads the out-half presence with the data: tests, repair A/B
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py" --rounds 2 repair128 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 128 --batch 256 --steps 5 --warmup 1 --pattern q3" new= prev=lib:celestia-app_amd/libdagpu_prev.so
