# Round-4 GPU experiments, one step per change (each: its GPU tests, then an
# interleaved A/B through tools/gpu_ab.sh).  Steps comparing against the previous
# build expect that build in celestia-app_amd/libdagpu_prev.so (make it from the
# parent commit; .so files are not in git).  Results: the profiles/*_r04.log named.
#   bash tools/gpu_r04.sh <step>
set -o pipefail
case "$1" in
  async)  # round 4: started Repairs (dagpu_repair_start / join) -- tests, then one batch vs 2 started slices (k = 128 and 512)
    mkdir -p gpurun_out
    timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_repair_async.py tests/test_gpu_repair_fill.py > gpurun_out/gpu_sub.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_sub.log
    [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 repair128 one= "slices2=args:--repair-slices 2" && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 512 --batch 4 --steps 4 --warmup 1" one= "slices2=args:--repair-slices 2"
    ;;
  dec512)  # round 4: GF(2^16) k = 512 decoder (two-group perms, paired-lane loads): tests, then A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py" --rounds 2 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  enc-merge)  # round 4: GF(2^16) encoder with the last IFFT / first FFT layers merged (no scratch): tests, A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py" --rounds 2 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  forest-multi)  # round 4: multi-level forest launches for the upper levels (forest_multi_kernel): tests, then split A/B by threshold
    bash tools/gpu_ab.sh --tests "tests/test_gpu_trees.py tests/test_gpu_split.py tests/test_gpu_proof.py tests/test_gpu_inclusion.py tests/test_gpu_c_client.py" --rounds 2 split512 m64= m32=DAGPU_FOREST_MULTI=32 m128=DAGPU_FOREST_MULTI=128 single=DAGPU_FOREST_MULTI=0
    ;;
  enc32)  # round 4: 32-elements-per-wave GF(2^16) encoders (leo16_encode_reg32_kernel, k = 256 and 512) vs 64 per wave: tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_repair_byz.py" --rounds 2 "bench:--mode split --split-k 256 --steps 10 --warmup 2" w32= w64=DAGPU_GF16_ENC32=0 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1 --pattern q3" w32= w64=DAGPU_GF16_ENC32=0 && \
    bash tools/gpu_ab.sh --rounds 1 split512 w32= w64=DAGPU_GF16_ENC32=0
    ;;
  dah)  # round 4: two-stage DAH for few wide squares (dah_sub_kernel + dah_top_kernel): tests, split A/B, then the stress profiles
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py tests/test_gpu_split.py tests/test_gpu_parity.py" --rounds 2 split512 dah2= dah1=DAGPU_DAH_SPLIT=0 && \
    bash tools/gpu_pmc_gf16.sh repair128 repair512 repair512q3 split512
    ;;
  split-pair)  # round 4: split slab forests in shared level launches (forest_enqueue_pair) and P = 1 without staging copies: tests, split A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_split.py tests/test_gpu_trees.py tests/test_gpu_bench_checks.py" --rounds 2 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode split --split-k 256 --steps 10 --warmup 2" new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  dec512-prefetch)  # round 4: k = 512 decoder with the next tables of a radix-4 unit loaded one phase ahead: tests, repair A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py" --rounds 3 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  fill-given)  # round 4: GF(2^16) fill encoders read the out-half presence before the transform (one ballot) instead of per element in the store loop: tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_gf16.py" --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1 --pattern q3" new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  gf8-fill-given)  # round 4: k = 128 sliced fill encoder reads the out-half presence with the data: tests, repair A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py" --rounds 2 repair128 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 128 --batch 256 --steps 5 --warmup 1 --pattern q3" new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  tables)  # round 4: decoder product tables from 16 gathers (e2 = 3 by XOR), logs from constants, none for unused tables: tests, A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_wide.py" --rounds 2 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  tables-first)  # round 4: k = 512 decoder issues its table gathers before the data loads (the barrier no longer waits for the data): tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py" --rounds 3 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  dec128-loads)  # round 4: k = 128 decoder issues its data loads before building the multiply tables: tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py" --rounds 3 repair128 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  col-maps)  # round 4: column presence-map kernels with more loads in flight (axis_complete_cols 16 waves, unrolled row loops): tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_gf16.py" --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 repair128 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  row-maps)  # round 4: row presence-map counts with 4 rows per wave (16 lanes per row): tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_gf16.py tests/test_gpu_repair_async.py" --rounds 2 repair128 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  dec512-tok)  # round 4: k = 512 decoder table loads ordered by tokens (new: each table during the previous phase, no SGPR spills; B: an intermediate build with tokens at unit ends only, 209 spills, not kept in git): tests, A/B
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_wide.py tests/test_gpu_repair_fill.py" --rounds 3 repair512 new= B=lib:celestia-app_amd/libdagpu_varB.so prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= B=lib:celestia-app_amd/libdagpu_varB.so prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  *) echo "steps: async dec512 enc-merge forest-multi enc32 dah split-pair dec512-prefetch fill-given gf8-fill-given tables tables-first dec128-loads col-maps row-maps dec512-tok"; exit 2;;
esac
