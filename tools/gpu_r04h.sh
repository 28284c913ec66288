# round 4: two-stage DAH for few wide squares (dah_sub_kernel + dah_top_kernel): tests, split A/B, then the stress profiles
set -o pipefail
bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py tests/test_gpu_split.py tests/test_gpu_parity.py" --rounds 2 split512 dah2= dah1=DAGPU_DAH_SPLIT=0 && \
bash tools/gpu_pmc_gf16.sh repair128 repair512 repair512q3 split512
