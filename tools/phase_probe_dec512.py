"""Phase timing of the k = 512 GF(2^16) decoder (leo16_decode_reg1k_kernel) from
a DAGPU_PHASE_PROBE build of the library: lane 0 of waves 0 and 15 of every
workgroup stamp s_memtime (shader clocks) at the phase boundaries; this prints
the mean clocks per phase over the workgroups of one Repair launch sequence.
    (build: make -C <copy of celestia-app_amd> libdagpu.so HIPFLAGS="... -DDAGPU_PHASE_PROBE",
     copy it to celestia-app_amd/libdagpu_probe.so)
    python tools/phase_probe_dec512.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DAGPU_LIB"] = os.path.join(ROOT, "celestia-app_amd", "libdagpu_probe.so")
for p in (ROOT, os.path.join(ROOT, "celestia-app_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from celestia_da import _abi, da  # noqa: E402

NAMES = ["tables built", "premultiply", "IFFT block (bits 0-5)", "transpose 1", "IFFT bits 6-9",
         "derivative", "FFT bits 9-6", "transpose 2", "FFT block (bits 5-0)", "postmultiply + stores"]
P = 12


def main():
    torch.cuda.set_device(0)
    ctx = da.Context(0)
    L = _abi.lib()
    L.dagpu_debug_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    bench.run_repair(ctx, 512, 2, 1, 1)  # warm
    torch.cuda.synchronize()
    L.dagpu_debug_probe(0, None, 0)
    bench.run_repair(ctx, 512, 2, 1, 0)
    torch.cuda.synchronize()
    n = 8192 * 2 * P
    buf = np.zeros(n, np.uint64)
    L.dagpu_debug_probe(1, buf.ctypes.data, n)
    st = buf.reshape(8192, 2, P).astype(np.int64)
    for wv, label in ((0, "wave 0"), (1, "wave 15")):
        s = st[:, wv, :]
        ok = (s[:, 0] > 0) & (s[:, 10] > 0)
        d = np.diff(s[ok][:, :11], axis=1)
        tot = (s[ok][:, 10] - s[ok][:, 0])
        print(f"{label}: {ok.sum()} workgroups stamped (the last launch's), mean total {tot.mean():.0f} clocks")
        for i, nm in enumerate(NAMES):
            print(f"  {nm:26s} {d[:, i].mean():9.0f}  ({100 * d[:, i].mean() / tot.mean():4.1f} %)")
    ctx.close()


if __name__ == "__main__":
    main()
