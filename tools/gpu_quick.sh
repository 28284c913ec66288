# quick GPU iteration: parity tests, bench (+ optional extra modes / microbench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in $*; do
  case $m in
    micro) timeout -k 10 120 ./tools/valu_bench > gpurun_out/valu_bench.log 2>&1 && cat gpurun_out/valu_bench.log || exit 1 ;;
    mixed|repair) timeout -k 10 300 python -u bench.py --mode $m --steps 5 --warmup 1 > gpurun_out/bench_$m.log 2>&1 && tail -1 gpurun_out/bench_$m.log || { tail -5 gpurun_out/bench_$m.log; exit 1; } ;;
  esac
done
