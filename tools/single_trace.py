"""Single-square drop-in latency probe (dagpu_extend_shares, the production
callers' shape: app/process_proposal.go:147-161).  Runs `calls` calls per mode
(roots only / EDS returned) at k and prints host-side latencies; run it under
`rocprofv3 --kernel-trace --memory-copy-trace` and summarise the last call of
each mode with tools/single_timeline.py.
usage: single_trace.py [k=128] [calls=10]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

from celestia_da import _abi, da, synth  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ctx = da.Context(0)
    L = ctx._L
    w = 2 * k
    src = da.PinnedBuffer(k * k * 512)
    src.array[:] = synth.blob_squares(k, 0xC0FFEE + k, 0, 1).reshape(-1)
    edsb = da.PinnedBuffer(w * w * 512)
    rr = np.empty(w * 90, np.uint8)
    cr = np.empty(w * 90, np.uint8)
    dah = np.empty(32, np.uint8)
    for mode, ptr in (("roots_only", 0), ("with_eds", edsb.ptr)):
        lat = []
        for _ in range(calls):
            t0 = time.perf_counter()
            rc = L.dagpu_extend_shares(ctx.handle, src.ptr, k * k, 512, ptr, _abi.addr(rr), _abi.addr(cr),
                                       _abi.addr(dah))
            lat.append((time.perf_counter() - t0) * 1e3)
            if rc:
                raise SystemExit(f"status {rc}")
        print(mode, " ".join(f"{x:.3f}" for x in lat), flush=True)
        time.sleep(0.05)  # a gap in the trace between the modes
    src.close()
    edsb.close()
    ctx.close()


if __name__ == "__main__":
    main()
