# Round-end GPU pass: parity suite, default bench (all config lines), repair kernel
# trace + decode-kernel PMC.  Outputs under gpurun_out/round/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/round; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit $rc; }
timeout -k 10 500 python -u bench.py > $OUT/bench_full.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench_full.log; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_repair -o run -- python3 bench.py --mode repair --steps 3 > $OUT/trace_repair.log 2>&1 || { echo "repair trace failed"; tail -5 $OUT/trace_repair.log; exit 1; }
echo "repair trace ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $OUT/pmc_repair_sq -o run -- python3 bench.py --mode repair --steps 2 --warmup 1 > $OUT/pmc_repair_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_repair_fetch -o run -- python3 bench.py --mode repair --steps 2 --warmup 1 > $OUT/pmc_repair_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_repair_write -o run -- python3 bench.py --mode repair --steps 2 --warmup 1 > $OUT/pmc_repair_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_repair_grbm -o run -- python3 bench.py --mode repair --steps 2 --warmup 1 > $OUT/pmc_repair_grbm.log 2>&1 || { echo "pmc grbm failed"; exit 1; }
echo "pmc ok"
