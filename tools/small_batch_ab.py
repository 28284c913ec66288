"""Device-resident small batches (n = 1 .. 16 squares at k): ms per
dagpu_extend_batch_device call, for choosing DAGPU_TREE_FUSED_MAX (the fused
per-tree NMT kernel vs one launch per tree level).  Run once per setting of the
variable (read once per process).  usage: small_batch_ab.py [k=128]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

from celestia_da import da, synth  # noqa: E402
from celestia_da.device import DeviceSquares  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    torch.cuda.set_device(0)
    ctx = da.Context(0)
    host = synth.blob_squares(k, 777, 0, 16)
    out = {}
    for n in (1, 2, 4, 8, 16):
        ds = DeviceSquares(k, n, device=0, ctx=ctx, in_place=True)
        ds.load_ods(host[:n])
        s = torch.cuda.current_stream()
        for _ in range(3):
            ds.extend(s)
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            ds.extend(s)
        torch.cuda.synchronize()
        out[n] = (time.perf_counter() - t0) / reps * 1e3
        want = [da.new_data_availability_header(da.extend_shares(host[i].reshape(k * k, 512), ctx)).hash()
                for i in range(n)]
        got = [bytes(ds.dah[i].cpu().numpy()) for i in range(n)]
        if got != want or (ds.status.cpu().numpy() != 0).any():
            raise SystemExit(f"n={n}: DAH mismatch")
        del ds
    print(os.environ.get("DAGPU_TREE_FUSED_MAX", "default"), k,
          " ".join(f"n={n}:{v:.3f}ms" for n, v in out.items()), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
