"""CPU tests: the oracle is pinned to the reference's golden vectors, cross-
checked against an independent pure-Python restatement, and reproduces the
committed fixtures.  (No GPU.)"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import pyref
from celestia_da import synth

from conftest import GOLDEN

FIX = json.load(open(os.path.join(GOLDEN, "squares.json")))
REF = FIX["reference"]


def _input(kind, k):
    if kind == "constant":
        return synth.constant_square(k)
    if kind == "tail_padding":
        return synth.tail_padding_square(k)
    raise ValueError(kind)


@pytest.mark.parametrize("portable", [False, True])
def test_sha256_matches_hashlib(portable):
    rng = np.random.default_rng(0)
    for n in list(range(0, 200)) + [542, 181, 91, 65, 1000]:
        msg = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.sha256(msg, portable=portable) == hashlib.sha256(msg).digest()


def test_gf8_tables_match_appendix():
    log, exp, skew, walsh = oracle.gf8_tables()
    # SURVEY.md Appendix A.1 first skew entries
    assert list(skew[:16]) == [255, 255, 85, 255, 17, 85, 34, 255, 153, 17, 102, 85, 51, 34, 187, 255]
    # exp/log are inverse permutations (log[0] = 255 sentinel)
    for a in range(1, 256):
        assert exp[log[a]] == a
    assert list(skew) == pyref.SKEW and list(log) == pyref.LOG


def test_nil_dah():
    # pkg/da/data_availability_header_test.go:15-25
    assert oracle.rfc6962_root([]).hex() == REF["nil_dah"]["hash"]


@pytest.mark.parametrize("name", ["min_dah", "typical_2x2", "max_128x128"])
def test_reference_golden_dah(name):
    case = REF[name]
    k = case["k"]
    ods = _input(case["input"], k)
    _, rr, cr, dah = oracle.extend_and_dah(ods, k, nthreads=8, want_eds=False)
    assert dah.hex() == case["hash"], case["src"]
    assert rr.shape == (2 * k, 90) and cr.shape == (2 * k, 90)  # root length 90 (malicious/app_test.go:60)


@pytest.mark.parametrize("k", [1, 2, 4])
def test_oracle_matches_pure_python(k):
    ods = synth.random_blob_square(k, 900 + k)
    eds, rr, cr, dah = oracle.extend_and_dah(ods, k)
    peds, prr, pcr, pdah = pyref.extend_and_dah([bytes(s) for s in ods], k)
    for r in range(2 * k):
        for c in range(2 * k):
            assert eds[r, c].tobytes() == peds[r][c]
    assert [bytes(x) for x in rr] == prr
    assert [bytes(x) for x in cr] == pcr
    assert dah == pdah


@pytest.mark.parametrize("k", [8, 16, 32, 64, 128])
def test_encode_matches_pure_python(k):
    rng = np.random.default_rng(k)
    data = rng.integers(0, 256, (k, 64), dtype=np.uint8)
    assert [bytes(p) for p in oracle.encode(data)] == pyref.encode([bytes(d) for d in data])


@pytest.mark.parametrize("case", FIX["random_blob"], ids=lambda c: f"k{c['k']}")
def test_fixture_random_blob(case):
    k = case["k"]
    ods = synth.random_blob_square(k, case["seed"])
    assert hashlib.sha256(ods.tobytes()).hexdigest() == case["ods_sha256"]
    eds, rr, cr, dah = oracle.extend_and_dah(ods, k, nthreads=8)
    assert hashlib.sha256(eds.tobytes()).hexdigest() == case["eds_sha256"]
    assert hashlib.sha256(rr.tobytes()).hexdigest() == case["row_roots_sha256"]
    assert hashlib.sha256(cr.tobytes()).hexdigest() == case["col_roots_sha256"]
    assert dah.hex() == case["dah"]


@pytest.mark.parametrize("case", FIX["codec"], ids=lambda c: f"k{c['k']}s{c['shard']}")
def test_fixture_codec(case):
    # regenerate the same sequential draws as make_fixtures.py
    rng = np.random.default_rng(7)
    for c in FIX["codec"]:
        data = rng.integers(0, 256, (c["k"], c["shard"]), dtype=np.uint8)
        if c is case:
            break
    assert hashlib.sha256(data.tobytes()).hexdigest() == case["data_sha256"]
    assert hashlib.sha256(oracle.encode(data).tobytes()).hexdigest() == case["parity_sha256"]


@pytest.mark.parametrize("k", [1, 2, 4, 8, 32, 128, 256])
def test_decode_roundtrip(k):
    """Leopard decode (GF(2^8); GF(2^16) at k=256 -- parity unpinned) inverts encode."""
    rng = np.random.default_rng(k + 5)
    d = rng.integers(0, 256, (k, 128), dtype=np.uint8)
    full = np.concatenate([d, oracle.encode(d)])
    for _ in range(3):
        pres = np.zeros(2 * k, bool)
        pres[rng.choice(2 * k, k, replace=False)] = True
        s = full.copy()
        s[~pres] = 0
        assert (oracle.decode(s, pres) == full).all()
    pres = np.zeros(2 * k, bool)
    pres[: k - 1] = True
    if k > 1:
        with pytest.raises(oracle.OracleError):
            oracle.decode(full, pres)


@pytest.mark.parametrize("k", [2, 4, 8, 16])
def test_q3_commutes(k):
    """specs data_structures.md:305-313: Q3 from rows of Q2 == from cols of Q1."""
    ods = synth.random_blob_square(k, 50 + k)
    eds = oracle.extend_square(ods, k)
    for c in range(k, 2 * k):
        assert (oracle.encode(np.ascontiguousarray(eds[:k, c])) == eds[k:, c]).all()


def test_push_order_violation():
    k = 4
    ods = synth.random_blob_square(k, 3)[::-1].copy()  # reverse order: unsorted namespaces
    with pytest.raises(oracle.OracleError) as e:
        oracle.extend_and_dah(ods, k)
    assert e.value.code == -4


@pytest.mark.parametrize("k", [2, 4, 8])
def test_repair_max_erasure(k):
    """C4 pattern: keep a random k x k sub-grid, erase the other 3k^2 cells."""
    rng = np.random.default_rng(k)
    ods = synth.random_blob_square(k, 77 + k)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k)
    w = 2 * k
    R = rng.choice(w, k, replace=False)
    C = rng.choice(w, k, replace=False)
    present = np.zeros((w, w), np.uint8)
    present[np.ix_(R, C)] = 1
    damaged = eds * present[:, :, None]
    rc, fixed = oracle.repair(damaged, present, k, rr, cr)
    assert rc == 0
    assert (fixed == eds).all()
    # byzantine: corrupt one present share -> ErrByzantineData
    bad = damaged.copy()
    bad[R[0], C[0], 100] ^= 1
    rc, _ = oracle.repair(bad, present, k, rr, cr)
    assert rc == -7
    # unrepairable: fewer than k per axis
    few = present.copy()
    few[R[0], :] = 0
    few[:, C[0]] = 0
    rc, _ = oracle.repair(damaged * few[:, :, None], few, k, rr, cr)
    assert rc == -6
