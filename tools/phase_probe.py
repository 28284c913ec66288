"""Phase timing of the Repair decoders from a DAGPU_PHASE_PROBE build of the
library: lane 0 of two waves of every workgroup stamps s_memtime (shader
clocks) at the phase boundaries; this prints the mean clocks per phase over the
workgroups of one Repair.
  dec512: leo16_decode_reg1k_kernel (k = 512, waves 0 and 15; DAGPU_DEC1K_PACKED=1)
  dec512h / dec256h / enc512h: the round-5 half-lane kernels
  dec128: leo8_decode128_sliced_kernel (k = 128, waves 0 and 3)
    (build: copy celestia-app_amd AND include/ side by side (the Makefile reads
     ../include/dagpu.h), make -C <copy>/celestia-app_amd libdagpu.so HIPFLAGS="... -DDAGPU_PHASE_PROBE",
     check `nm -D` shows dagpu_debug_probe, copy it to celestia-app_amd/libdagpu_probe.so)
    python tools/phase_probe.py [dec512|dec128]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DAGPU_LIB", os.path.join(ROOT, "celestia-app_amd", "libdagpu_probe.so"))
for p in (ROOT, os.path.join(ROOT, "celestia-app_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from celestia_da import _abi, da  # noqa: E402

KERNELS = {
    "dec512": dict(fn="dagpu_debug_probe", P=12, k=512, n=2, waves=("wave 0", "wave 15"),
                   names=["tables built", "premultiply", "IFFT block (bits 0-5)", "transpose 1", "IFFT bits 6-9",
                          "derivative", "FFT bits 9-6", "transpose 2", "FFT block (bits 5-0)",
                          "postmultiply + stores"]),
    # round 5: the half-lane GF(2^16) kernels (rs_gf16.hip H_PROBE; op 1 = decoder stamps, op 2 = encoder)
    "dec512h": dict(fn="dagpu_debug_probe", op=1, P=14, k=512, n=2, waves=("wave 0", "wave 15"),
                    names=["tables, loads", "premultiply", "IFFT bit 0 (S) + swap", "IFFT bits 1-5 (B)",
                           "transpose 1", "IFFT bits 6-9 (T)", "derivative", "FFT bits 9-6 (T)", "transpose 2",
                           "FFT bits 5-1 (B)", "swap + FFT bit 0 (S)", "postmultiply + stores"]),
    "dec256h": dict(fn="dagpu_debug_probe", op=1, P=14, k=256, n=8, waves=("wave 0", "wave 7"),
                    names=["tables, loads", "premultiply", "IFFT bit 0 (S) + swap", "IFFT bits 1-5 (B)",
                           "transpose 1", "IFFT bits 6-8 (T)", "derivative", "FFT bits 8-6 (T)", "transpose 2",
                           "FFT bits 5-1 (B)", "swap + FFT bit 0 (S)", "postmultiply + stores"]),
    "enc512h": dict(fn="dagpu_debug_probe", op=2, P=14, split=512, waves=("wave 0", "wave 7"),
                    names=["loads (+ copy, given)", "IFFT bit 0 (S) + swap", "IFFT bits 1-5 (B)", "transpose 1",
                           "IFFT 6-7, merged 8, FFT 7-6 (T)", "transpose 2", "FFT bits 5-1 (B)",
                           "swap + FFT bit 0 (S)", "stores"]),
    "dec128": dict(fn="dagpu_debug_probe8", P=14, k=128, n=256, waves=("wave 0", "wave 3"),
                   names=["tables, loads, premultiply, transpose8", "IFFT layers 0-1 (A)", "transpose A->A*",
                          "IFFT layers 2-3 (A*)", "exchange A*->B", "IFFT layers 4-7 (B)", "derivative",
                          "FFT layers 7-4 (B)", "exchange B->A*", "FFT layers 3-2 (A*)", "barrier + A*->A",
                          "FFT layers 1-0 (A)", "transpose8, postmultiply, stores"]),
}


def main():
    kern = KERNELS[sys.argv[1] if len(sys.argv) > 1 else "dec512"]
    P, names = kern["P"], kern["names"]
    last = len(names)
    torch.cuda.set_device(0)
    ctx = da.Context(0)
    L = _abi.lib()
    fn = getattr(L, kern["fn"])
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    if "split" in kern:  # the split square at P = 1 (its row and column encodes)
        bench.bench_split(None, 0, 1, 0, ctx, kern["split"], 1, 1)
        torch.cuda.synchronize()
        fn(0, None, 0)
        bench.bench_split(None, 0, 1, 0, ctx, kern["split"], 1, 0)
    else:
        bench.run_repair(ctx, kern["k"], kern["n"], 1, 1)  # warm
        torch.cuda.synchronize()
        fn(0, None, 0)
        bench.run_repair(ctx, kern["k"], kern["n"], 1, 0)
    torch.cuda.synchronize()
    n = 8192 * 2 * P
    buf = np.zeros(n, np.uint64)
    fn(kern.get("op", 1), buf.ctypes.data, n)
    st = buf.reshape(8192, 2, P).astype(np.int64)
    for wv, label in enumerate(kern["waves"]):
        s = st[:, wv, :]
        ok = (s[:, 0] > 0) & (s[:, last] > 0)
        d = np.diff(s[ok][:, :last + 1], axis=1)
        tot = (s[ok][:, last] - s[ok][:, 0])
        print(f"{label}: {ok.sum()} workgroups stamped (the last launch's), mean total {tot.mean():.0f} clocks")
        for i, nm in enumerate(names):
            print(f"  {nm:38s} {d[:, i].mean():9.0f}  ({100 * d[:, i].mean() / tot.mean():4.1f} %)")
    ctx.close()


if __name__ == "__main__":
    main()
