#!/bin/bash
# Rehearse bench.py's N>1 path (sharded headline, block replay with the DAH
# all-gather, split stress with the all-to-all) on a ONE-GPU box: every rank on
# GPU 0, collectives over gloo (DAGPU_BENCH_SHARED_GPU=1).  Not scaling numbers.
set -euo pipefail
mkdir -p gpurun_out
export DAGPU_BENCH_SHARED_GPU=1
for n in 2 4; do
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 --no-configs \
    --distinct 16 --replay-blocks 2048 > gpurun_out/rehearse_n$n.log 2>&1
  tail -c 3000 gpurun_out/rehearse_n$n.log
done
