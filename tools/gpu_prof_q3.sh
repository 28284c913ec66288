# Kernel stats of the Q3-only repair (reverse fill) and of configs[3] on the final build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pq3; mkdir -p $OUT
for spec in "128 256 q3" "128 256 subgrid" "512 2 q3"; do
  set -- $spec
  L=k$1_$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$L -o run -- python3 bench.py --mode repair --k $1 --batch $2 --pattern $3 --steps 3 --warmup 1 > $OUT/$L.log 2>&1 || { echo "trace $L failed"; tail -5 $OUT/$L.log; exit 1; }
  echo "== $L"; tail -1 $OUT/$L.log | cut -c1-160
  s=$(find $OUT/$L -name "*kernel_stats.csv" | head -1)
  cp "$s" $OUT/kernel_stats_$L.csv
  cut -d, -f1-4 "$s" | grep dagpu | head -12
done
