# Round 6, last session: GPU steps after the wide-codec / k = 16384 split work.
# A/B steps expect celestia-app_amd/libdagpu_base.so built beforehand on the CPU
# (tools/build_variant.sh base <rev>); delete it after the call.
#   bash tools/gpu_r06b.sh <step>
set -o pipefail
mkdir -p gpurun_out
case "$1" in
  ab)  # node_to_rec per dword (split k = 512), wide-kernel templates (k = 2048 Repair / split), codec timings
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_split16k.py > gpurun_out/r06b_ab_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06b_ab_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 40 --warmup 3" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode split --split-k 2048 --steps 4 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    timeout -k 10 300 python -u tools/codec_wide.py 3 > gpurun_out/r06b_codec_wide.log 2>&1 && cat gpurun_out/r06b_codec_wide.log && \
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_codec -o codec -- python3 -u tools/codec_wide.py 2 > gpurun_out/r06b_codec_prof.log 2>&1
    ;;
esac
case "$1" in
  slices)  # started-repair slices for the Repair lines (C4 k = 128 x 256, k = 512 x 2)
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 128 --batch 256 --steps 10 --warmup 2" s1= s2=args:--repair-slices\ 2 s4=args:--repair-slices\ 4 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 512 --batch 2 --steps 10 --warmup 2" s1= s2=args:--repair-slices\ 2
    ;;
  slices8)  # more slices for C4
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode repair --k 128 --batch 256 --steps 10 --warmup 2" s1= s4=args:--repair-slices\ 4 s8=args:--repair-slices\ 8 s16=args:--repair-slices\ 16
    ;;
esac
case "$1" in
  w2)  # k = 2048 decoder: 8-symbol slices at 512 threads (two workgroups per CU) vs 16 at 1,024 (one)
        # (historical: the DAGPU_WIDE4096_NG2 switch was removed after this A/B lost; profiles/wide2048_ng2_ab_r06.log)
    DAGPU_LIB=celestia-app_amd/libdagpu_w2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "k2048 or decode_matches or codec_beyond" > gpurun_out/r06b_w2_tests.log 2>&1
    rc=$?; echo "w2 tests rc=$rc"; tail -2 gpurun_out/r06b_w2_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 2048 --batch 1 --steps 3 --warmup 1" new= w2=lib:celestia-app_amd/libdagpu_w2.so
    ;;
esac
case "$1" in
  init)  # fused Repair start-up (one init launch, known[] from the completeness kernels) + roots queued ahead of the deferred-axis read
        # (historical: the change was reverted after this A/B, within noise; profiles/repair_init_ab_r06.log)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_parity.py tests/test_gpu_gf16.py > gpurun_out/r06b_init_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06b_init_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 128 --batch 256 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
esac
case "$1" in
  slices_n)  # C4: started-repair slice counts around 4
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode repair --k 128 --batch 256 --steps 10 --warmup 2" s1= s3=args:--repair-slices\ 3 s4=args:--repair-slices\ 4 s5=args:--repair-slices\ 5 s6=args:--repair-slices\ 6
    ;;
esac
case "$1" in
  roots2)  # Repair verification: the second half's roots on a side stream behind the first half's leaves
        # (historical: reverted after this A/B; profiles/repair_roots2_ab_r06.log)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_gf16.py tests/test_gpu_parity.py > gpurun_out/r06b_roots2_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06b_roots2_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "repair or k4096" > gpurun_out/r06b_roots2_wide.log 2>&1
    rc=$?; echo "wide rc=$rc"; tail -2 gpurun_out/r06b_roots2_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode repair --k 512 --batch 2 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 512 --batch 2 --steps 10 --warmup 2 --pattern q3" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 1024 --batch 2 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
esac
