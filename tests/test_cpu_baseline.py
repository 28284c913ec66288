"""The SIMD CPU baseline (oracle/da_simd.c, bench.py cpu_baseline "simd-port")
computes exactly what the scalar oracle computes: EDS bytes, all row/column
roots and the DAH, for random blob squares k = 1..128 and the reference's
golden 2x2 / 128x128 constant squares (pkg/da/data_availability_header_test.go:43-54),
at 1 and several threads; a push-order violation is reported the same way."""
import json
import os

import numpy as np
import pytest

import oracle
from celestia_da import synth

from conftest import GOLDEN

REF = json.load(open(os.path.join(GOLDEN, "squares.json")))["reference"]


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128])
def test_simd_matches_oracle(k):
    ods = synth.blob_squares(k, 77, k, 1)[0].reshape(k * k, 512)
    oeds, orr, ocr, odah = oracle.extend_and_dah(ods, k, nthreads=8)
    sq = oracle.SimdSquare(k)
    for threads in (1, 5):
        eds, rr, cr, dah = sq.run(ods, threads)
        assert (eds == oeds).all()
        assert (rr == orr).all() and (cr == ocr).all()
        assert dah == odah


@pytest.mark.parametrize("name", ["typical_2x2", "max_128x128"])
def test_simd_golden(name):
    case = REF[name]
    k = case["k"]
    _, _, _, dah = oracle.SimdSquare(k).run(synth.constant_square(k), 4)
    assert dah.hex() == case["hash"], case["src"]


def test_simd_push_order():
    k = 8
    ods = synth.random_blob_square(k, 9)[::-1].copy()
    with pytest.raises(oracle.OracleError) as e:
        oracle.SimdSquare(k).run(ods, 2)
    assert e.value.code == -4


def test_simd_isa_named():
    assert "SHA-256" in oracle.simd_isa()
