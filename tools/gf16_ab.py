"""A/B of the GF(2^16) kernels (k = 256 / 512: register-resident rs_gf16.hip
vs the LDS-slice kernels of rs_gf16_wide.hip, DAGPU_GF16_WIDE=1) on the
configs[4] stress workloads, interleaved in one process: one square through
the split path at P = 1 (ms per square), Repair with the maximal erasure
pattern (random sub-grid and Q3 kept; squares/s), plus the wide-only widths
(k = 1024, 2048) for reference.

    python tools/gf16_ab.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "celestia-app_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
from celestia_da import da  # noqa: E402


def one(ctx, k, what):
    if what == "split":
        r = bench.bench_split(None, 0, 1, 0, ctx, k, 3, 1)
        return {"ms_per_square": round(r["ms_per_square"], 4), "dah_ok": r["dah_matches_single_gpu"]}
    nsq = {256: 8, 512: 2, 1024: 1, 2048: 1}[k]
    pattern = "q3" if what == "repair_q3" else "subgrid"
    r = bench.run_repair(ctx, k, nsq, 2, 1, pattern=pattern)
    return {"squares_per_s": round(r["squares_per_s"], 2), "bit_exact": r["bit_exact"]}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    torch.cuda.set_device(0)
    ctx = da.Context(0)
    out = {}
    for r in range(rounds):
        for k in (256, 512):
            for wide in ("0", "1"):
                os.environ["DAGPU_GF16_WIDE"] = wide
                for what in ("split", "repair", "repair_q3"):
                    res = one(ctx, k, what)
                    out.setdefault(f"k{k} {what} wide={wide}", []).append(res)
                    print(f"round {r} k={k} {what} wide={wide}: {res}", flush=True)
        os.environ.pop("DAGPU_GF16_WIDE", None)
        if r == 0:
            for k, whats in ((1024, ("split", "repair", "repair_q3")), (2048, ("repair",))):
                for what in whats:
                    res = one(ctx, k, what)
                    out.setdefault(f"k{k} {what}", []).append(res)
                    print(f"k={k} {what}: {res}", flush=True)
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
