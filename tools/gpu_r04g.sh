# round 4: 32-elements-per-wave GF(2^16) encoders (leo16_encode_reg32_kernel, k = 256 and 512) vs 64 per wave: tests, A/B
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_repair_byz.py" --rounds 2 "bench:--mode split --split-k 256 --steps 10 --warmup 2" w32= w64=DAGPU_GF16_ENC32=0 && \
bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1 --pattern q3" w32= w64=DAGPU_GF16_ENC32=0 && \
bash tools/gpu_ab.sh --rounds 1 split512 w32= w64=DAGPU_GF16_ENC32=0
