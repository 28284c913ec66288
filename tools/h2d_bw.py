"""Host->device copy bandwidth for the drop-in (PCIe) mode: one 512 MiB pinned
batch (64 k=128 ODS) copied as 1, 2, 4 or 8 chunks on as many streams, and a
pull by a device kernel (torch copy from a pinned tensor mapped into the GPU
address space).  Prints one JSON line per variant."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    n = 64 * 128 * 128 * 512
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    host.random_(0, 255)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    back = torch.empty(64 * 512 * 2 * 90, dtype=torch.uint8).pin_memory()
    for chunks in (1, 2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(chunks)]
        step = n // chunks

        def go():
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    dev[i * step:(i + 1) * step].copy_(host[i * step:(i + 1) * step], non_blocking=True)
        t = timed(go)
        print(json.dumps({"variant": f"h2d_{chunks}_streams", "GBps": n / t / 1e9}), flush=True)
    for mib in (8, 32, 256):  # one EDS (k=64: 8 MiB, k=128: 32 MiB) back to pinned memory
        m = mib << 20
        t = timed(lambda: host[:m].copy_(dev[:m], non_blocking=True))
        print(json.dumps({"variant": f"d2h_{mib}MiB_pinned", "GBps": m / t / 1e9, "ms": t * 1e3}), flush=True)
    t = timed(lambda: back.copy_(dev[:back.numel()], non_blocking=True))
    print(json.dumps({"variant": "d2h_roots_batch", "GBps": back.numel() / t / 1e9, "ms": t * 1e3}), flush=True)


if __name__ == "__main__":
    main()
