#!/bin/bash
# Rehearse bench.py's N>1 path (sharded headline, block replay with the DAH
# all-gather, split stress k = 256 / 512 with the all-to-all, the per-rank
# report) on a ONE-GPU box: every rank on GPU 0, collectives over gloo
# (DAGPU_BENCH_SHARED_GPU=1).  Code-path check, not scaling numbers.
#   bash tools/gpu_rehearse_multi.sh [ranks...]   (default 2 4 8)
set -euo pipefail
mkdir -p gpurun_out
export DAGPU_BENCH_SHARED_GPU=1
for n in ${@:-2 4 8}; do
  timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 --no-configs \
    --batch 64 --distinct 16 --replay-blocks 2048 --split-k 256 512 > gpurun_out/rehearse_n$n.log 2>&1
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
t = open(f"gpurun_out/rehearse_n{n}.log").read()
d = json.loads(t[t.index('{"metric"'):].splitlines()[0])
br = d.get("block_replay", {})
split = {k: v.get("dah_matches_single_gpu") for k, v in d.get("split_stress", {}).items()}
print(f"ranks {n}: value {d['value']:.0f} squares/s, headline_bit_exact {d.get('headline_bit_exact')}, "
      f"replay bit_exact {br.get('bit_exact')}, split dah_matches_single_gpu {split}, "
      f"step_ms {d['ranks']['step_ms']}, transport {d['ranks']['transport']}")
PY
done
