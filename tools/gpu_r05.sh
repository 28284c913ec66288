# Round-5 GPU steps (each: its GPU tests, then an interleaved A/B through
# tools/gpu_ab.sh).  Steps comparing against the previous build expect it in
# celestia-app_amd/libdagpu_prev.so (built from the parent commit; .so files are
# not in git).  Results: the profiles/*_r05.log named in DESIGN.md.
#   bash tools/gpu_r05.sh <step>
set -o pipefail
mkdir -p gpurun_out
case "$1" in
  base)  # round 5 start: new tests (started-repair structure, k = 1024 chunked DAH, k = 4096 / 8192 squares), default bench, stress counters
    timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_repair_async.py tests/test_gpu_wide.py > gpurun_out/r05_base_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_base_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 400 python -u bench.py > gpurun_out/r05_base_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r05_base_bench.log; exit 1; }
    bash tools/gpu_pmc_gf16.sh repair512 split512 repair128
    ;;
  mul332)  # round 5: GF(2^16) multiply with a 3/3/2 bit split (12 v_perm per 4 symbols instead of 16), units layer by layer: tests, A/B vs the previous build
    bash tools/gpu_ab.sh --tests "tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_wide.py tests/test_gpu_repair_byz.py" --rounds 2 split512 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" new= prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512 new= prev=lib:celestia-app_amd/libdagpu_prev.so
    ;;
  first)  # round 5 first GPU pass: correctness of everything new (3/3/2 multiply, half-lane k = 512 decoder, started-repair fixes, wide squares), then A/Bs
    timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_async.py tests/test_gpu_wide.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_first_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_first_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 repair512 new= packed=DAGPU_DEC1K_PACKED=1 prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 split512 new= reg32=DAGPU_GF16_ENCH=0 prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512q3 new= reg32=DAGPU_GF16_ENCH=0 prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_pmc_gf16.sh repair512 split512
    ;;
  pf)  # round 5: k = 256 half-lane kernels and the SGPR table prefetch (issued one group ahead): tests, A/B vs the build without prefetch (nopf) and round 4 (prev)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_split.py > gpurun_out/r05_pf_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_pf_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 repair512 new= nopf=lib:celestia-app_amd/libdagpu_nopf.so && \
    bash tools/gpu_ab.sh --rounds 2 split512 new= nopf=lib:celestia-app_amd/libdagpu_nopf.so prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 repair512q3 new= nopf=lib:celestia-app_amd/libdagpu_nopf.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" new= nopf=lib:celestia-app_amd/libdagpu_nopf.so prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1 --pattern q3" new= nopf=lib:celestia-app_amd/libdagpu_nopf.so prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 256 --steps 10 --warmup 2" new= nopf=lib:celestia-app_amd/libdagpu_nopf.so prev=lib:celestia-app_amd/libdagpu_prev.so && \
    bash tools/gpu_pmc_gf16.sh repair512 split512
    ;;
  probe)  # round 5: phase probes of the half-lane kernels (libdagpu_probe.so, a -DDAGPU_PHASE_PROBE build), then the whole suite + default bench
    for w in dec512h dec256h enc512h; do
      timeout -k 10 300 python -u tools/phase_probe.py $w > gpurun_out/phase_probe_${w}_r05.log 2>&1 || { echo "probe $w failed"; tail -5 gpurun_out/phase_probe_${w}_r05.log; exit 1; }
      cat gpurun_out/phase_probe_${w}_r05.log
    done
    bash tools/gpu_final.sh
    ;;
  skip)  # round 5: half-lane decoders skip the loads of missing shards (out-of-range voffset): tests, A/B vs DAGPU_DEC_LOADALL=1
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py > gpurun_out/r05_skip_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_skip_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 skip= all=DAGPU_DEC_LOADALL=1 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" skip= all=DAGPU_DEC_LOADALL=1
    ;;
  splitov)  # round 5: forest levels fold all-parity waves, uniform forests upload nothing (no host syncs in the split
            # steps), split column encode on a side stream beside the leaves of rows 0..k-1: tests, then A/B
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_trees.py tests/test_gpu_inclusion.py tests/test_gpu_proof.py > gpurun_out/r05_splitov_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_splitov_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 50 --warmup 5" ov1= ov0=DAGPU_SPLIT_OVERLAP=0 ov2=DAGPU_SPLIT_OVERLAP=2 head=lib:celestia-app_amd/libdagpu_head.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 20 --warmup 3" ov1= ov0=DAGPU_SPLIT_OVERLAP=0 head=lib:celestia-app_amd/libdagpu_head.so
    ;;
  dectab)  # round 5: half-lane decoders build ONE 3/3/2 table per element (pre for present, post for missing): tests, A/B
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_dectab_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_dectab_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 tab= head=lib:celestia-app_amd/libdagpu_head.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" tab= head=lib:celestia-app_amd/libdagpu_head.so
    ;;
  zskip)  # round 5: butterflies at zero skews (positions 2^m - 1) skip their multiply (half-lane T layers, wide kernels)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_split.py > gpurun_out/r05_zskip_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_zskip_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_wide.py -k "not k8192 and not k4096" > gpurun_out/r05_zskip_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r05_zskip_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 zs= tab=lib:celestia-app_amd/libdagpu_tab.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" zs= tab=lib:celestia-app_amd/libdagpu_tab.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 zs= tab=lib:celestia-app_amd/libdagpu_tab.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 512 --steps 50 --warmup 5" zs= tab=lib:celestia-app_amd/libdagpu_tab.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 2 --warmup 1" zs= tab=lib:celestia-app_amd/libdagpu_tab.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" zs= tab=lib:celestia-app_amd/libdagpu_tab.so
    ;;
  probe2)  # round 5: phase probes of the half-lane kernels after the one-table / zero-skew changes (libdagpu_probe.so rebuilt)
    for w in dec512h dec256h enc512h; do
      timeout -k 10 300 python -u tools/phase_probe.py $w > gpurun_out/phase_probe_${w}_r05b.log 2>&1 || { echo "probe $w failed"; tail -5 gpurun_out/phase_probe_${w}_r05b.log; exit 1; }
      cat gpurun_out/phase_probe_${w}_r05b.log
    done
    ;;
  load64)  # round 5: half-lane decoders load lane pairs with 8-byte loads + a DPP swap (half the VMEM instructions)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_load64_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_load64_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 l64= l32=DAGPU_DEC_LOAD32=1 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" l64= l32=DAGPU_DEC_LOAD32=1 && \
    bash tools/gpu_pmc_gf16.sh repair512 split512 split1024 repair1024
    ;;
  enc64)  # round 5: half-lane encoders' loads, Q0 copy and plain / fill stores as 8-byte lane-pair accesses (env A/B);
          # wide decoder: one product table per element instead of log/exp gathers per symbol (A/B vs libdagpu_zs.so)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_split.py tests/test_gpu_parity.py > gpurun_out/r05_enc64_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_enc64_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_wide.py -k "not k8192" > gpurun_out/r05_enc64_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r05_enc64_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 2 --warmup 1" wd= zs=lib:celestia-app_amd/libdagpu_zs.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 1 --warmup 1" wd= zs=lib:celestia-app_amd/libdagpu_zs.so && \
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 50 --warmup 5" e64= e32=DAGPU_ENC_LOAD32=1 && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 e64= e32=DAGPU_ENC_LOAD32=1 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 256 --steps 50 --warmup 5" e64= e32=DAGPU_ENC_LOAD32=1
    ;;
  colorder)  # round 5: the split's column push-order flag into its one status word (was a per-tree slot past it)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_trees.py tests/test_gpu_inclusion.py tests/test_gpu_proof.py tests/test_gpu_parity.py > gpurun_out/r05_colorder_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_colorder_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_colorder_tests.log | head; exit $rc; }
    ;;
  order)  # round 5: half-lane decoders issue their table gathers, then the data loads, then pack the table
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_order_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_order_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 ord= ord0=lib:celestia-app_amd/libdagpu_ord0.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" ord= ord0=lib:celestia-app_amd/libdagpu_ord0.so
    ;;
  order8)  # round 5: the k = 128 sliced decoder issues its table loads, presence bytes and shard data before the table barrier
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_parity.py tests/test_gpu_repair_async.py > gpurun_out/r05_order8_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_order8_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair128 ord= ord0=lib:celestia-app_amd/libdagpu_ord0.so
    ;;
  der64)  # round 5: the half-lane decoders' derivative stages lo and hi side by side (8-byte LDS accesses)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_der64_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_der64_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 d64= d0=lib:celestia-app_amd/libdagpu_der0.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" d64= d0=lib:celestia-app_amd/libdagpu_der0.so
    ;;
  wide2048)  # round 5: kernel stats + SQ/GRBM counters of the k = 2048 split square and Repair (wide kernels)
    bash tools/gpu_pmc_gf16.sh split2048 repair2048
    ;;
  wtab)  # round 5: wide kernels load wave-uniform skew tables with scalar loads (radix-4 steps with dist * CH >= 64)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_wide.py -k "not k8192" > gpurun_out/r05_wtab_wide.log 2>&1
    rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/r05_wtab_wide.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 1024 --steps 10 --warmup 2" ws= w0=lib:celestia-app_amd/libdagpu_w0.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 1024 --batch 1 --steps 2 --warmup 1" ws= w0=lib:celestia-app_amd/libdagpu_w0.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode repair --k 2048 --batch 1 --steps 1 --warmup 1" ws= w0=lib:celestia-app_amd/libdagpu_w0.so && \
    bash tools/gpu_ab.sh --rounds 1 "bench:--mode split --split-k 2048 --steps 2 --warmup 1" ws= w0=lib:celestia-app_amd/libdagpu_w0.so
    ;;
  vtab)  # round 5: the decoders' dist-2 B layers read their skew tables with vector loads (no VGPR copies of SGPR pools)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py > gpurun_out/r05_vtab_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_vtab_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 repair512 vt= lb0=lib:celestia-app_amd/libdagpu_lb0.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 256 --batch 8 --steps 5 --warmup 1" vt= lb0=lib:celestia-app_amd/libdagpu_lb0.so
    ;;
  onepart)  # round 5: the split at one part passes its own records to the finish (no gather copies; the A/B switch was removed after this run)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_bench_checks.py > gpurun_out/r05_onepart_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_onepart_tests.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 20 --warmup 3" new= old=DAGPU_SPLIT_GATHER=1
    ;;
  sqpath)  # round 5: one-part split below k = 1024 through the square pipeline's roots kernels (DAGPU_SPLIT_SQUARE=0: forests)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_split.py > gpurun_out/r05_sqpath_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_sqpath_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_sqpath_tests.log | head; exit $rc; }
    bash tools/gpu_ab.sh --rounds 3 "bench:--mode split --split-k 512 --steps 20 --warmup 3" sq= forest=DAGPU_SPLIT_SQUARE=0 && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode split --split-k 256 --steps 20 --warmup 3" sq= forest=DAGPU_SPLIT_SQUARE=0
    ;;
  slices)  # round 5: the headline's RS/NMT pipeline slice count and first-slice size, re-checked on the final kernels
    bash tools/gpu_ab.sh --rounds 2 headline s4= s6=DAGPU_PIPE_SLICES=6 s8=DAGPU_PIPE_SLICES=8 f32=DAGPU_PIPE_FIRST=32 f48=DAGPU_PIPE_FIRST=48
    ;;
  fillskip)  # round 5: Repair rounds launch a fill direction only when the plan put vectors in it (and size pair grids by count)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_repair_fill.py tests/test_gpu_repair_byz.py tests/test_gpu_repair_async.py tests/test_gpu_parity.py tests/test_gpu_gf16.py > gpurun_out/r05_fillskip_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_fillskip_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05_fillskip_tests.log | head; exit $rc; }
    bash tools/gpu_ab.sh --rounds 2 repair512 fs= fe0=lib:celestia-app_amd/libdagpu_fe0.so && \
    bash tools/gpu_ab.sh --rounds 2 repair512q3 fs= fe0=lib:celestia-app_amd/libdagpu_fe0.so && \
    bash tools/gpu_ab.sh --rounds 2 repair128 fs= fe0=lib:celestia-app_amd/libdagpu_fe0.so && \
    bash tools/gpu_ab.sh --rounds 2 "bench:--mode repair --k 128 --batch 256 --steps 3 --warmup 1 --pattern q3" fs= fe0=lib:celestia-app_amd/libdagpu_fe0.so
    ;;
  final-a)  # round end, part 1: the whole -m gpu suite, the default bench line and its rocprofv3 kernel trace
    bash tools/gpu_final.sh
    ;;
  final-b)  # round end, part 2: headline counters (kernel stats + FETCH/WRITE/SQ/GRBM passes, --no-check) and the stress / wide counters
    bash tools/gpu_profile.sh r05 counters && \
    bash tools/gpu_pmc_gf16.sh repair512 repair512q3 split512 repair128 split1024 repair1024
    ;;
  *) echo "steps: base mul332 first pf probe skip splitov dectab zskip probe2 load64 enc64 colorder order order8 der64 wide2048 wtab final-a final-b"; exit 2;;
esac
