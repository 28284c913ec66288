# Kernel-trace stats of the GF(2^16) stress workloads (k = 512 Repair, random
# sub-grid and Q3 kept; the split square k = 512 at P = 1), one rocprofv3 run each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_gf16; mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 bench.py "$@" \
    > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; return 1; }
  f=$(find $OUT/$name -name "*kernel_stats.csv" | head -1)
  echo "== $name"; head -12 "$f" | cut -d, -f1-8
}
run repair512 --mode repair --k 512 --batch 2 --steps 3 --warmup 1 && \
run repair512q3 --mode repair --k 512 --batch 2 --steps 3 --warmup 1 --pattern q3 && \
run split512 --mode split --split-k 512 --steps 3 --warmup 1
