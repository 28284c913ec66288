"""A/B of the single-square drop-in latency (bench.py bench_single, the
ProcessProposal shape) over environment switches of the library, in one
process with the variants interleaved (the library reads them per call).
Round 4 used it for the row-slab upload and fused tree-top experiments
(profiles/single_square_ab_r04.log; both removed).

    python tools/single_square.py [rounds] [VAR=a,b ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "celestia-app_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import bench  # noqa: E402
from celestia_da import da  # noqa: E402


def variants(args):
    """VAR=a,b -> one variant per value ('auto' = unset); no args: the default build."""
    out = {"default": {}}
    for a in args:
        key, vals = a.split("=", 1)
        out = {f"{n} {key}={v}".strip(): dict(env, **{key: v}) for n, env in out.items() for v in vals.split(",")}
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = da.Context(0)
    out = {}
    for r in range(rounds):
        for name, env in variants(sys.argv[2:]).items():
            for key, v in env.items():
                if v == "auto":
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = v
            res = bench.bench_single(ctx, ks=(64, 128), calls=60, trace=True)
            for k, rk in res.items():
                for mode in ("roots_only", "with_eds"):
                    m = rk[mode]
                    out.setdefault(name, {}).setdefault(f"k{k}_{mode}", []).append(
                        {"p50": round(m["p50_ms"], 4), "p99": round(m["p99_ms"], 4),
                         "stages": m.get("stages_median_ms")})
            print(f"round {r} {name}: " + ", ".join(
                f"k{k} {mode} p50 {res[k][mode]['p50_ms']:.3f}" for k in res for mode in ("roots_only", "with_eds")),
                flush=True)
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
