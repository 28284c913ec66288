# Round-6 GPU steps.  Steps comparing against another build expect it built
# beforehand on the CPU with tools/build_variant.sh (e.g. `base HEAD` ->
# celestia-app_amd/libdagpu_base.so, or a -D variant); delete it after the call
# (.so files are not in git).  Results: the profiles/*_r06*.log named in DESIGN.md.
# (The `tail` step's switch DAGPU_NMT_TAIL was removed with the kernel it chose.)
#   bash tools/gpu_r06.sh <step>
set -o pipefail
mkdir -p gpurun_out
case "$1" in
  clean)  # round 6 start: the tree without the retired kernels/switches -- whole GPU suite, default bench
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_clean_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_clean_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u bench.py > gpurun_out/r06_clean_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r06_clean_bench.log; exit 1; }
    tail -c 600 gpurun_out/r06_clean_bench.log
    ;;
  fillskip)  # round 6: fill-candidate counts from the count launch; fill launches skipped on axes without candidates
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_parity.py tests/test_gpu_bench_checks.py > gpurun_out/r06_fillskip_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_fillskip_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_fillskip_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_fillskip_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair128 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
  q2ke)  # round 6: quarter-lane k = 2048 encoder (16 waves, one workgroup per CU) vs the wide one
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192" > gpurun_out/r06_q2ke_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_q2ke_wide.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_split.py > gpurun_out/r06_q2ke_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_q2ke_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 2048 --steps 4 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1 --pattern q3" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
  tail)  # round 6: fused NMT tree tail (few squares in flight) vs one launch per level
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_repair_fill.py tests/test_gpu_square.py tests/test_gpu_proof.py > gpurun_out/r06_tail_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_tail_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 30 --warmup 3" new= off=DAGPU_NMT_TAIL=0 base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 headline new= base=lib:celestia-app_amd/libdagpu_base.so && \
    timeout -k 10 300 python -u tools/single_square.py 3 DAGPU_NMT_TAIL=auto,0 > gpurun_out/r06_tail_single.log 2>&1 && tail -12 gpurun_out/r06_tail_single.log
    ;;
  q1kc)  # round 6: k = 1024 decoder without the S-layer offset spill; counters of the k >= 1024 kernels
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_q1kc_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_q1kc_wide.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py > gpurun_out/r06_q1kc_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_q1kc_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_pmc_gf16.sh repair1024 split1024 repair2048
    ;;
  q1ke)  # round 6: quarter-lane k = 1024 encoder (8 waves, two workgroups per CU) + decoder vs HEAD (quarter decoder, wide encoder)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_q1ke_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_q1ke_wide.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_parity.py > gpurun_out/r06_q1ke_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_q1ke_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1 --pattern q3" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 512 --steps 30 --warmup 3" new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
  q1k)  # round 6: quarter-lane k = 1024 decoder (16 waves, one workgroup per CU) vs the wide one
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_q1k_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_q1k_wide.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py > gpurun_out/r06_q1k_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_q1k_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" new= wide=DAGPU_GF16_WIDE=1 base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 1024 --batch 2 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 512 --batch 2 --steps 5 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so
    ;;
  ctl)  # round 6: Repair round control -- fused count/mark launches, mailbox counters, early candidate heads
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_parity.py tests/test_gpu_gf16.py tests/test_gpu_c_client.py > gpurun_out/r06_ctl_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_ctl_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_ctl_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_ctl_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair128 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_repair_timeline.sh repair512 repair128
    ;;
  dec1)  # round 6: per-pattern decoder tables (glds), double-buffered transposes, LDS bit-0 tables (decoder + encoder)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_split.py > gpurun_out/r06_dec1_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_dec1_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_dec1_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_dec1_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 512 --steps 30 --warmup 3" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" new= base=lib:celestia-app_amd/libdagpu_base.so && \
    for w in dec512h enc512h; do
      for v in probe probebase; do
        DAGPU_LIB=celestia-app_amd/libdagpu_$v.so timeout -k 10 300 python -u tools/phase_probe.py $w > gpurun_out/phase_probe_${w}_${v}_r06.log 2>&1 || { echo "probe $w $v failed"; tail -5 gpurun_out/phase_probe_${w}_${v}_r06.log; exit 1; }
        echo "== $w $v"; cat gpurun_out/phase_probe_${w}_${v}_r06.log | grep -v amdgpu.ids
      done
    done
    ;;
  dec2)  # round 6: quarter-lane k = 512 decoder (two workgroups per CU) vs the half-lane one (round-6 form) vs round 5
    timeout -k 10 60 ./tools/permlane_check > gpurun_out/r06_permlane.log 2>&1; echo "permlane rc=$?"; head -c 1200 gpurun_out/r06_permlane.log
    DAGPU_LIB=celestia-app_amd/libdagpu_q.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r06_dec2_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_dec2_tests.log; [ $rc -eq 0 ] || exit $rc
    DAGPU_LIB=celestia-app_amd/libdagpu_q.so timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r06_dec2_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r06_dec2_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 q=lib:celestia-app_amd/libdagpu_q.so half=lib:celestia-app_amd/libdagpu_half.so base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" q=lib:celestia-app_amd/libdagpu_q.so base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1" q=lib:celestia-app_amd/libdagpu_q.so base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" q=lib:celestia-app_amd/libdagpu_q.so base=lib:celestia-app_amd/libdagpu_base.so
    ;;
  dec3)  # round 6: quarter-lane k = 512 encoder (four workgroups per CU) vs the half-lane one; counters of the new kernels
    DAGPU_LIB=celestia-app_amd/libdagpu_qe.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_split.py > gpurun_out/r06_dec3_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_dec3_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 qe=lib:celestia-app_amd/libdagpu_qe.so he=lib:celestia-app_amd/libdagpu_he.so && \
    bash tools/gpu_ab.sh --rounds 3 repair512q3 qe=lib:celestia-app_amd/libdagpu_qe.so he=lib:celestia-app_amd/libdagpu_he.so base=lib:celestia-app_amd/libdagpu_base.so && \
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 30 --warmup 3" qe=lib:celestia-app_amd/libdagpu_qe.so he=lib:celestia-app_amd/libdagpu_he.so base=lib:celestia-app_amd/libdagpu_base.so && \
    DAGPU_LIB=celestia-app_amd/libdagpu_qe.so bash tools/gpu_pmc_gf16.sh repair512 repair512q3 split512 repair1024 repair2048
    ;;
  val1)  # round 6: the whole tree -- every GPU test, the default bench line and its trace, the headline counters
    bash tools/gpu_final.sh && bash tools/gpu_profile.sh r06 counters
    ;;
  val2)  # round 6: k = 256 quarter-lane decoder and 1,024-thread wide kernels (A/B), then the whole tree
    DAGPU_LIB=celestia-app_amd/libdagpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gf16.py > gpurun_out/r06_val2_gf16.log 2>&1
    rc=$?; echo "gf16 tests rc=$rc"; tail -2 gpurun_out/r06_val2_gf16.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 10 --warmup 2" q256= h256=lib:celestia-app_amd/libdagpu_h256.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 3 --warmup 1" w1024= w512=lib:celestia-app_amd/libdagpu_w512.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 2 --warmup 1" w1024= w512=lib:celestia-app_amd/libdagpu_w512.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" w1024= w512=lib:celestia-app_amd/libdagpu_w512.so && \
    bash tools/gpu_final.sh
    ;;
  *) echo "unknown step $1"; exit 2;;
esac
