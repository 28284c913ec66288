"""Experiment: RS/SHA overlap by slicing a 256-square k=128 batch into S groups,
RS of every group on stream R and the NMT/DAH work of group i on stream H
after RS(i) (so RS(i+1..) can run beside the hashing of group i).  ODS in
place (Q0 of the EDS buffer).  Prints ms per 256 squares for each S and stream
priority setting (argument nmt_hi: the hashing stream at high priority
instead), and checks the DAHs against the unsliced run."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "celestia-app_amd"))
from celestia_da import da, synth  # noqa: E402
from celestia_da.device import DeviceSquares  # noqa: E402

k, B = 128, 256
ctx = da.Context(0)
host = synth.blob_squares(k, 77, 0, B)
ref = DeviceSquares(k, B, ctx=ctx, in_place=True)
ref.load_ods(host)
ref.extend()
torch.cuda.synchronize()
want = ref.dah.cpu()
del ref
torch.cuda.empty_cache()


def run(S, prio, nmt_hi=False):
    groups = [DeviceSquares(k, B // S, ctx=ctx, in_place=True) for _ in range(S)]
    for i, g in enumerate(groups):
        g.load_ods(host[i * (B // S):(i + 1) * (B // S)])
    lo, hi = torch.cuda.Stream.priority_range()
    sr = torch.cuda.Stream(priority=hi if prio else 0)
    sh = torch.cuda.Stream(priority=hi if nmt_hi else 0)
    evs = [torch.cuda.Event() for _ in range(S)]
    torch.cuda.synchronize()

    def step():
        cur = torch.cuda.current_stream()
        sr.wait_stream(cur)
        sh.wait_stream(cur)
        for i, g in enumerate(groups):
            g.extend_rs(sr)
            evs[i].record(sr)
        for i, g in enumerate(groups):
            sh.wait_event(evs[i])
            g.roots(sh)
        cur.wait_stream(sh)
        cur.wait_stream(sr)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 20
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    got = torch.cat([g.dah.cpu() for g in groups])
    ok = bool(torch.equal(got, want))
    print(f"S={S} prio={int(prio)} nmt_hi={int(nmt_hi)}: {ms:.3f} ms/256 squares  {B / ms * 1e3:.0f} squares/s  dah_ok={ok}", flush=True)
    del groups
    torch.cuda.empty_cache()


modes = sys.argv[1:] or ["all"]
for S in (1, 2, 4, 8):
    if "nmt_hi" in modes:
        if S > 1:
            run(S, False)
            run(S, False, nmt_hi=True)
        continue
    for prio in ((False, True) if S > 1 else (False,)):
        run(S, prio)
