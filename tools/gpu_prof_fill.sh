# Kernel stats of the repair bench (k = 128 and k = 512) with the fill route on and off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pfill; mkdir -p $OUT
for kb in "128 256" "512 2"; do
  set -- $kb
  for f in 1 0; do
    DAGPU_REPAIR_FILL=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$1f$f -o run -- python3 bench.py --mode repair --k $1 --batch $2 --steps 3 --warmup 1 > $OUT/k$1f$f.log 2>&1 || { echo "trace $1 $f failed"; tail -5 $OUT/k$1f$f.log; exit 1; }
    echo "== k=$1 fill=$f"; tail -1 $OUT/k$1f$f.log | cut -c1-160
    s=$(find $OUT/k$1f$f -name "*kernel_stats.csv" | head -1)
    cut -d, -f1-4 "$s" | grep dagpu | head -16
  done
done
