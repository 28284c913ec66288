"""Drop-in (PCIe) pipeline variants for bench.py's end_to_end figure: pinned
host ODS -> H2D -> extend -> D2H roots + DAH, 64 k=128 squares per batch.
  two_streams   : bench.py's original (copies and kernels of a batch on one stream, 2 buffers)
  copy_stream   : all H2D on one dedicated stream, kernels + D2H on a compute stream,
                  events between them, N buffers
Prints one JSON line per variant."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "celestia-app_amd"))
from celestia_da import da  # noqa: E402
from celestia_da.device import DeviceSquares  # noqa: E402

K, B = 128, 64


def make_bufs(ctx, n):
    w = 2 * K
    out = []
    for _ in range(n):
        ds = DeviceSquares(K, B, device=0, ctx=ctx)
        o = {"rr": torch.empty((B, w, 90), dtype=torch.uint8).pin_memory(),
             "cr": torch.empty((B, w, 90), dtype=torch.uint8).pin_memory(),
             "dah": torch.empty((B, 32), dtype=torch.uint8).pin_memory()}
        out.append((ds, o))
    return out


def run_two_streams(ctx, pin, steps):
    bufs = make_bufs(ctx, 2)
    sts = [torch.cuda.Stream() for _ in range(2)]

    def one(i):
        (ds, o), st = bufs[i % 2], sts[i % 2]
        with torch.cuda.stream(st):
            ds.ods.copy_(pin, non_blocking=True)
            ds.extend(st)
            o["rr"].copy_(ds.row_roots, non_blocking=True)
            o["cr"].copy_(ds.col_roots, non_blocking=True)
            o["dah"].copy_(ds.dah, non_blocking=True)
    return timed(one, steps)


def run_copy_stream(ctx, pin, steps, nbuf):
    bufs = make_bufs(ctx, nbuf)
    cs, ks = torch.cuda.Stream(), torch.cuda.Stream()
    loaded = [torch.cuda.Event() for _ in range(nbuf)]
    freed = [torch.cuda.Event() for _ in range(nbuf)]
    used = [False] * nbuf

    def one(i):
        j = i % nbuf
        ds, o = bufs[j]
        with torch.cuda.stream(cs):
            if used[j]:
                cs.wait_event(freed[j])
            ds.ods.copy_(pin, non_blocking=True)
            loaded[j].record(cs)
        with torch.cuda.stream(ks):
            ks.wait_event(loaded[j])
            ds.extend(ks)
            o["rr"].copy_(ds.row_roots, non_blocking=True)
            o["cr"].copy_(ds.col_roots, non_blocking=True)
            o["dah"].copy_(ds.dah, non_blocking=True)
            freed[j].record(ks)
        used[j] = True
    return timed(one, steps)


def timed(one, steps):
    for i in range(2):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(2, 2 + steps):
        one(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ctx = da.Context(0)
    rng = np.random.default_rng(0)
    ods = rng.integers(0, 256, (B, K * K, 512), dtype=np.uint8)
    ods[:, :, :29] = 0  # one namespace: push order holds
    pin = torch.from_numpy(ods.reshape(B, -1)).pin_memory()
    steps = 12
    tag = os.environ.get("E2E_TAG", "")
    t = run_two_streams(ctx, pin, steps)
    print(json.dumps({"variant": "two_streams" + tag, "ms_per_batch": t * 1e3, "squares_per_s": B / t}), flush=True)
    for nbuf in (2, 3):
        t = run_copy_stream(ctx, pin, steps, nbuf)
        print(json.dumps({"variant": f"copy_stream_{nbuf}buf" + tag, "ms_per_batch": t * 1e3,
                          "squares_per_s": B / t}), flush=True)


if __name__ == "__main__":
    main()
