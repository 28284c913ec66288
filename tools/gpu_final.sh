# Round-end GPU pass: the whole -m gpu suite, the default bench line, and the
# rocprofv3 kernel-trace summary of that same default bench command.
# Outputs under gpurun_out/final/ (copy the summaries into profiles/).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit $rc; }
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
echo "bench ok"; grep '^{"metric"' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('headline_bit_exact'))"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_default -o run -- python3 bench.py > $OUT/trace_default.log 2>&1 || { echo "default-bench trace failed"; tail -5 $OUT/trace_default.log; exit 1; }
echo "default-bench trace ok"
