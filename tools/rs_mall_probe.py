"""How much would the RS column pass gain from reading Q0|Q1 out of the
Infinity Cache (MALL, 256 MB) instead of HBM?  Times the row and column passes
(dagpu_profile_enable brackets, one launch each) for batches of n k=128
squares: at n <= 8 the batch's Q0|Q1 (16 MiB per square) stays MALL-resident
between the row pass and the column pass (and across repeats), at n >= 32 it
does not.  Prints per-square microseconds per pass."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from celestia_da import _abi, da, synth  # noqa: E402
from celestia_da.device import DeviceSquares  # noqa: E402

os.environ["DAGPU_PIPE_SLICES"] = "1"
ctx = da.Context(0)
L = ctx._L
k = 128
res = {}
for n in (2, 4, 8, 16, 32, 64, 128, 256):
    ds = DeviceSquares(k, n, ctx=ctx, in_place=True)
    ds.load_ods(synth.blob_squares(k, 77, 0, min(n, 16), threads=16)[np.arange(n) % min(n, 16)])
    reps = max(4, 512 // n)
    for _ in range(3):
        ds.extend_rs()
    torch.cuda.synchronize()
    L.dagpu_profile_enable(ctx.handle, 1)
    L.dagpu_profile_read(ctx.handle, None, None, 1)
    for _ in range(reps):
        ds.extend_rs()
    torch.cuda.synchronize()
    L.dagpu_profile_enable(ctx.handle, 0)
    tot = np.zeros(len(_abi.PROFILE_KERNELS))
    cnt = np.zeros(len(_abi.PROFILE_KERNELS), np.uint64)
    L.dagpu_profile_read(ctx.handle, _abi.addr(tot), _abi.addr(cnt), 1)
    row, col = tot[0] / cnt[0], tot[1] / cnt[1]
    res[n] = {"row_us_per_sq": row * 1e3 / n, "col_us_per_sq": col * 1e3 / n,
              "col_TBps_actual": n * 16 * 2**20 * 2 / (col * 1e-3) / 1e12}
    print(n, json.dumps(res[n]), flush=True)
    del ds
    torch.cuda.empty_cache()
