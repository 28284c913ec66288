"""Codec throughput past the square widths (dagpu_encode / dagpu_decode at
k = 8192, 16384, 32768; include/dagpu.h DAGPU_MAX_CODEC_WIDTH).  Host buffers
(the rsmt2d.Codec boundary), so wall times include PCIe; run under
`rocprofv3 --kernel-trace --stats` for the kernels' own times.
    python tools/codec_wide.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "celestia-app_amd"))
from celestia_da import _abi, da  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = da.Context(0)
    rng = np.random.default_rng(7)
    for k, nvec in ((8192, 16), (16384, 8), (32768, 4)):
        shard = 512
        data = rng.integers(0, 256, (nvec, k, shard), dtype=np.uint8)
        par = np.empty_like(data)
        ctx.check(ctx._L.dagpu_encode(ctx.handle, k, nvec, shard, _abi.addr(data), _abi.addr(par)))
        t = time.perf_counter()
        for _ in range(reps):
            ctx.check(ctx._L.dagpu_encode(ctx.handle, k, nvec, shard, _abi.addr(data), _abi.addr(par)))
        te = (time.perf_counter() - t) / reps
        full = np.concatenate([data, par], axis=1)
        pres = np.zeros((nvec, 2 * k), np.uint8)
        for v in range(nvec):
            pres[v, rng.choice(2 * k, k, replace=False)] = 1
        damaged = np.ascontiguousarray(full * pres[:, :, None])
        buf = damaged.copy()
        ctx.check(ctx._L.dagpu_decode(ctx.handle, k, nvec, shard, _abi.addr(buf), _abi.addr(pres)))
        assert (buf == full).all()
        t = time.perf_counter()
        for _ in range(reps):
            buf[:] = damaged
            ctx.check(ctx._L.dagpu_decode(ctx.handle, k, nvec, shard, _abi.addr(buf), _abi.addr(pres)))
        td = (time.perf_counter() - t) / reps
        mib = nvec * k * shard / 2**20
        print(f"k={k} nvec={nvec} shard={shard}: encode {te * 1e3:.2f} ms ({mib:.0f} MiB data), "
              f"decode {td * 1e3:.2f} ms (k of 2k kept, {2 * mib:.0f} MiB shards), bit-exact", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
