# round 3, first GPU pass: full -m gpu suite, k=512/k=128 repair A/B against
# the round-2 library, the D2H path probe (plus its kernel trace), and a short
# bench with the single-square stage timelines.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
fi
for spec in "n512::--k 512 --batch 2" "p512:DAGPU_LIB=celestia-app_amd/libdagpu_prev.so:--k 512 --batch 2" \
            "n128::--k 128 --batch 256" "p128:DAGPU_LIB=celestia-app_amd/libdagpu_prev.so:--k 128 --batch 256"; do
  label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
  env $envs timeout -k 10 300 python -u bench.py --mode repair --steps 5 --warmup 1 $args > gpurun_out/rep_$label.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/rep_$label.log; exit $rc; fi
  echo "$label $(tail -1 gpurun_out/rep_$label.log | cut -c1-200)"
done
timeout -k 10 120 ./tools/d2h_probe 16 > gpurun_out/d2h_probe.log 2>&1 || { echo d2h_probe failed; cat gpurun_out/d2h_probe.log; exit 1; }
cat gpurun_out/d2h_probe.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/d2h_prof -o d2h -- $GRAFT_REPO_ROOT/tools/d2h_probe 16 > $GRAFT_REPO_ROOT/gpurun_out/d2h_prof.log 2>&1; echo "d2h prof rc=$?"; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-replay --no-configs > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.log
