# kernel-trace stats of the repair and mixed benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; mkdir -p $OUT
for m in repair mixed; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$m -o run -- python3 bench.py --mode $m --steps 3 --warmup 1 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
done
echo ok
