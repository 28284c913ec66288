"""Experiment: overlap of RS (memory/VALU) and SHA (VALU) by running batch
slices on S HIP streams.  Prints ms per 64-square step for S = 1, 2, 4."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "celestia-app_amd"))
from celestia_da import da, synth  # noqa: E402
from celestia_da.device import DeviceSquares  # noqa: E402

k = 128
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = da.Context(0)
host = np.stack([synth.random_blob_square(k, i).reshape(-1) for i in range(8)])
for S in (1, 2, 4, 8):
    groups = [DeviceSquares(k, B // S, ctx=ctx) for _ in range(S)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    for g in groups:
        for i in range(g.n):
            g.ods[i].copy_(torch.from_numpy(host[i % 8]))
    torch.cuda.synchronize()
    for mode in ("fused", "staged"):
        def step():
            if mode == "fused":
                for g, s in zip(groups, streams):
                    g.extend(s)
            else:  # RS of all groups first, then roots, each on its own stream
                for g, s in zip(groups, streams):
                    g.extend_rs(s)
                for g, s in zip(groups, streams):
                    g.roots(s)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        print(f"S={S} {mode}: {ms:.3f} ms/step  {B / ms * 1e3:.0f} squares/s", flush=True)
    del groups
    torch.cuda.empty_cache()
