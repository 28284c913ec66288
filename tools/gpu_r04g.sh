# round 4: 16-wave k = 512 GF(2^16) encoder (leo16_encode_reg16_kernel) vs the 8-wave one: tests, A/B
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_repair_byz.py" --rounds 2 split512 w16= w8=DAGPU_GF16_ENC16=0 && \
bash tools/gpu_ab.sh --rounds 2 repair512q3 w16= w8=DAGPU_GF16_ENC16=0
