# round 4: split slab forests in shared level launches (forest_enqueue_pair) and P = 1 without staging copies: tests, split A/B vs the previous build
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_split.py tests/test_gpu_trees.py tests/test_gpu_bench_checks.py" --rounds 2 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
bash tools/gpu_ab.sh --rounds 1 "bench:--mode split --split-k 256 --steps 10 --warmup 2" new= prev=lib:celestia-app_amd/libdagpu_prev.so
