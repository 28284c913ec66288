set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/split -o run -- python3 bench.py --mode split --steps 3 --warmup 1 > $OUT/split.log 2>&1 || { tail -20 $OUT/split.log; exit 1; }
find $OUT/split -name "*stats*" | head
