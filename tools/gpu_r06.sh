# Round-6 GPU steps.  Steps comparing against another build expect it in
# celestia-app_amd/libdagpu_ab_<label>.so (deleted again after the call; .so
# files are not in git).  Results: the profiles/*_r06*.log named in DESIGN.md.
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
  *) echo "unknown step $1"; exit 2;;
esac
