"""Generate tests/golden/squares.json (committed fixtures).

Two kinds of vectors:
  * "reference": hashes copied from the reference's own tests (the parity
    anchors), with the file:line they come from.  Inputs are the reference's
    deterministic generators (constant shares, tail padding).
  * "oracle": regression vectors produced by the CPU oracle (oracle/da_oracle.c)
    on seeded random-namespace blob squares (celestia_da.synth).  The oracle is
    pinned by the "reference" vectors; the Go reference itself cannot run here
    (no Go toolchain, modules not vendored -- SURVEY.md §8c), so these are the
    oracle's outputs, not the reference's.

Run:  python tests/golden/make_fixtures.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import oracle  # noqa: E402
from celestia_da import synth  # noqa: E402

REFERENCE = {
    "nil_dah": {
        "src": "pkg/da/data_availability_header_test.go:15-25",
        "hash": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
    },
    "min_dah": {
        "src": "pkg/da/data_availability_header_test.go:27-32",
        "k": 1,
        "input": "tail_padding",
        "hash": "3d96b7d238e7e0456f6af8e7cdf0a67bd6cf9c2089ecb559c659dcaa1f880353",
    },
    "typical_2x2": {
        "src": "pkg/da/data_availability_header_test.go:43-48",
        "k": 2,
        "input": "constant",
        "hash": "b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25",
    },
    "max_128x128": {
        "src": "pkg/da/data_availability_header_test.go:49-54",
        "k": 128,
        "input": "constant",
        "hash": "0bd3abeeacfbb0b92dfbdac4a154868e3c4e79666f7fcf6c620bb90dd3a0dcf0",
    },
}

SEEDS = {1: 101, 2: 102, 4: 104, 8: 108, 16: 116, 32: 132, 64: 164, 128: 228}


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def main() -> None:
    out = {"reference": REFERENCE, "random_blob": [], "codec": []}
    for k, seed in SEEDS.items():
        ods = synth.random_blob_square(k, seed)
        eds, rr, cr, dah = oracle.extend_and_dah(ods, k, nthreads=8)
        case = {
            "k": k,
            "seed": seed,
            "ods_sha256": sha(ods.tobytes()),
            "eds_sha256": sha(eds.tobytes()),
            "row_roots_sha256": sha(rr.tobytes()),
            "col_roots_sha256": sha(cr.tobytes()),
            "dah": dah.hex(),
        }
        if k <= 8:
            case["row_roots"] = [bytes(r).hex() for r in rr]
            case["col_roots"] = [bytes(r).hex() for r in cr]
            case["eds_row_sha256"] = [sha(eds[r].tobytes()) for r in range(2 * k)]
        out["random_blob"].append(case)
    rng = np.random.default_rng(7)
    for k in (1, 2, 4, 8, 16, 32, 64, 128):
        for shard in (64, 512):
            data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
            par = oracle.encode(data)
            out["codec"].append({
                "k": k, "shard": shard, "data_sha256": sha(data.tobytes()),
                "parity_sha256": sha(par.tobytes()), "rng": "default_rng(7) sequential",
            })
    with open(os.path.join(HERE, "squares.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "squares.json"))


if __name__ == "__main__":
    main()
