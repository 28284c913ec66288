# Instruction-cache counters for the k=128 encode kernel (tools/rs_bench2.cpp build "rsb_base").
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/icache; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|SQ_BUSY_CU_CYCLES\|SQ_INSTS_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt || true
cat $OUT/names.txt | tr '\n' ' '; echo
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/p1 -o run -- "$GRAFT_REPO_ROOT/tools/rsb_base" base > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail -5 $OUT/p1.log; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d $OUT/p2 -o run -- "$GRAFT_REPO_ROOT/tools/rsb_base" base > $OUT/p2.log 2>&1 || { echo "p2 failed"; tail -5 $OUT/p2.log; }
echo done
