"""GPU parity tests: the HIP path (through the C ABI) against the reference's
golden vectors, the committed fixtures and the CPU oracle on identical inputs.
Integer/byte work: every comparison is bit-exact."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from celestia_da import _abi, da, synth

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(GOLDEN, "squares.json")))
REF = FIX["reference"]


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


# --- reference golden vectors (pkg/da/data_availability_header_test.go) -------

def test_min_data_availability_header(ctx):
    dah = da.min_data_availability_header(ctx)
    assert dah.hash().hex() == REF["min_dah"]["hash"]
    dah.validate_basic()


@pytest.mark.parametrize("name", ["typical_2x2", "max_128x128"])
def test_new_data_availability_header_golden(ctx, name):
    case = REF[name]
    k = case["k"]
    eds = da.extend_shares(synth.constant_square(k), ctx)
    got = da.new_data_availability_header(eds)
    assert len(got.row_roots) == 2 * k and len(got.column_roots) == 2 * k
    assert got.hash().hex() == case["hash"], case["src"]
    # memoised Hash equals the host-side RFC-6962 recomputation
    assert da.DataAvailabilityHeader(got.row_roots, got.column_roots).hash() == got.hash()


def test_nil_hash():
    assert da.nil_dah_hash().hex() == REF["nil_dah"]["hash"]


# --- committed fixtures -------------------------------------------------------

@pytest.mark.parametrize("case", FIX["random_blob"], ids=lambda c: f"k{c['k']}")
def test_fixture_squares(ctx, case):
    k = case["k"]
    ods = synth.random_blob_square(k, case["seed"])
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    assert sha(eds.data.tobytes()) == case["eds_sha256"]
    assert sha(b"".join(dah.row_roots)) == case["row_roots_sha256"]
    assert sha(b"".join(dah.column_roots)) == case["col_roots_sha256"]
    assert dah.hash().hex() == case["dah"]


# --- oracle on fresh seeded inputs ---------------------------------------------

@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128])
def test_extend_matches_oracle(ctx, k):
    for seed in (k * 31 + 1, k * 31 + 2):
        ods = synth.random_blob_square(k, seed)
        eds = da.extend_shares(ods, ctx)
        dah = da.new_data_availability_header(eds)
        oeds, orr, ocr, odah = oracle.extend_and_dah(ods, k, nthreads=8)
        assert (eds.data == oeds).all()
        assert b"".join(dah.row_roots) == orr.tobytes()
        assert b"".join(dah.column_roots) == ocr.tobytes()
        assert dah.hash() == odah


@pytest.mark.parametrize("k", [1, 4, 32])
def test_tail_padding_and_parity_namespace_edge(ctx, k):
    # Q0 made only of tail padding / shares whose namespace IS the parity
    # namespace: exercises the ignoreMaxNamespace branch of HashNode.
    for ods in (synth.tail_padding_square(k), np.full((k * k, 512), 0xFF, np.uint8)):
        eds = da.extend_shares(ods, ctx)
        dah = da.new_data_availability_header(eds)
        _, orr, ocr, odah = oracle.extend_and_dah(ods, k)
        assert b"".join(dah.row_roots) == orr.tobytes()
        assert b"".join(dah.column_roots) == ocr.tobytes()
        assert dah.hash() == odah


def test_mixed_parity_namespace_tail(ctx):
    # sorted random blob shares followed by shares carrying the parity namespace
    k = 8
    ods = synth.random_blob_square(k, 5)
    ods[-5:, :29] = 0xFF
    ods = synth.sort_shares(ods)
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    _, orr, ocr, odah = oracle.extend_and_dah(ods, k)
    assert dah.hash() == odah and b"".join(dah.row_roots) == orr.tobytes()


def test_push_order_violation(ctx):
    k = 8
    ods = synth.random_blob_square(k, 9)[::-1].copy()
    eds = da.extend_shares(ods, ctx)  # ExtendShares itself succeeds (rsmt2d)
    with pytest.raises(da.ErrInvalidPushOrder):
        da.new_data_availability_header(eds)
    with pytest.raises(oracle.OracleError):
        oracle.extend_and_dah(ods, k)
    # single swapped adjacent pair inside one row / one column
    for (a, b) in ((0, 1), (0, k)):
        ods = synth.random_blob_square(k, 10)
        ods[[a, b]] = ods[[b, a]]
        eds = da.extend_shares(ods, ctx)
        with pytest.raises(da.ErrInvalidPushOrder):
            da.new_data_availability_header(eds)


def test_extend_batch_mixed_k(ctx):
    rng = np.random.default_rng(3)
    ks = [int(2 ** rng.integers(0, 8)) for _ in range(24)]
    ods = [synth.random_blob_square(k, 500 + i) for i, k in enumerate(ks)]
    eds, rr, cr, dah, status = da.extend_batch(np.concatenate([o.reshape(-1) for o in ods]), ks, ctx,
                                               want_eds=True)
    assert (status == 0).all()
    off = 0
    for i, k in enumerate(ks):
        oeds, orr, ocr, odah = oracle.extend_and_dah(ods[i], k, nthreads=8)
        n = 4 * k * k * 512
        assert (eds[off:off + n] == oeds.reshape(-1)).all()
        off += n
        assert (rr[i] == orr).all() and (cr[i] == ocr).all()
        assert dah[i].tobytes() == odah


def test_extend_batch_pipelined(ctx, monkeypatch):
    """Host mode splits a large uniform batch into chunks: H2D of chunk c on the
    copy stream while chunk c-1 is extended (dagpu.cpp run_group_pipelined).
    Many small chunks (chunk override) and the default 16-square chunks at
    k=128 must give what the single-shot path gives; a push-order violation in
    a middle chunk is reported for that square only."""
    k, n = 8, 37
    ods = np.stack([synth.random_blob_square(k, 900 + i).reshape(-1) for i in range(n)])
    ods[20].reshape(k * k, 512)[[0, 1]] = ods[20].reshape(k * k, 512)[[1, 0]]
    monkeypatch.setenv("DAGPU_PIPELINE_CHUNK", "100000")
    ref = da.extend_batch(ods.reshape(-1), [k] * n, ctx, want_eds=True)
    monkeypatch.setenv("DAGPU_PIPELINE_CHUNK", "5")
    got = da.extend_batch(ods.reshape(-1), [k] * n, ctx, want_eds=True)
    got2 = da.extend_batch(ods.reshape(-1), [k] * n, ctx, want_eds=False)
    assert (got[0] == ref[0]).all()
    for a, b in ((got[1], ref[1]), (got[2], ref[2]), (got2[1], ref[1])):
        assert all((x == y).all() for x, y in zip(a, b))
    assert (got[3] == ref[3]).all() and (got2[3] == ref[3]).all()
    assert list(np.nonzero(got[4])[0]) == [20] and (got[4] == ref[4]).all()
    _, orr, ocr, odah = oracle.extend_and_dah(ods[36], k)
    assert got[3][36].tobytes() == odah
    monkeypatch.delenv("DAGPU_PIPELINE_CHUNK")
    k, n = 128, 40  # default chunk: 16 squares (128 MiB) -> 3 chunks
    host = np.stack([synth.random_blob_square(k, 8000 + (i % 5)).reshape(-1) for i in range(n)])
    _, _, _, hdah, st = da.extend_batch(host.reshape(-1), [k] * n, ctx)
    assert (st == 0).all()
    for i in range(5):
        _, _, _, odah = oracle.extend_and_dah(host[i], k, nthreads=8, want_eds=False)
        assert all(hdah[j].tobytes() == odah for j in range(i, n, 5))


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128])
@pytest.mark.parametrize("shard", [64, 512, 1536])
def test_codec_encode_matches_oracle(ctx, k, shard):
    rng = np.random.default_rng(k * shard)
    data = rng.integers(0, 256, (3, k, shard), dtype=np.uint8)
    par = da.LeoRSCodec(ctx).encode_batch(data)
    for v in range(3):
        assert (par[v] == oracle.encode(data[v])).all()


@pytest.mark.parametrize("k", [16, 32, 64, 128])
@pytest.mark.parametrize("shard", [512, 1024])
def test_codec_encode_sliced_shapes(ctx, k, shard):
    """Vector counts that are multiples of 4 and whole 512-B chunks take the
    bit-sliced kernel (rs_gf8_sliced.hip) through the codec entry too."""
    rng = np.random.default_rng(k + shard)
    data = rng.integers(0, 256, (8, k, shard), dtype=np.uint8)
    par = da.LeoRSCodec(ctx).encode_batch(data)
    for v in range(8):
        assert (par[v] == oracle.encode(data[v])).all()


_PACKED_CHILD = r"""
import hashlib, sys
sys.path[:0] = sys.argv[1:3]
from celestia_da import _abi, da, synth
ctx = da.Context(0)
for k in (16, 32, 64, 128):
    eds = da.extend_shares(synth.random_blob_square(k, 100 + k), ctx)
    print(k, hashlib.sha256(eds.data.tobytes()).hexdigest())
ctx.close()
"""


def test_packed_and_sliced_encoders_agree(ctx):
    """The packed-byte encoder (DAGPU_ENC_SLICED=0, read once per process, so
    in a child process) and the default bit-sliced encoder give the same EDS."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DAGPU_ENC_SLICED="0")
    out = subprocess.run([sys.executable, "-c", _PACKED_CHILD, os.path.join(root, "celestia-app_amd"),
                          os.path.join(root, "oracle")], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    packed = dict(line.split() for line in out.stdout.split("\n") if line.strip() and line.split()[0].isdigit())
    assert len(packed) == 4
    for k in (16, 32, 64, 128):
        eds = da.extend_shares(synth.random_blob_square(k, 100 + k), ctx)
        assert sha(eds.data.tobytes()) == packed[str(k)], k


def test_codec_fixture(ctx):
    rng = np.random.default_rng(7)
    codec = da.LeoRSCodec(ctx)
    for c in FIX["codec"]:
        data = rng.integers(0, 256, (c["k"], c["shard"]), dtype=np.uint8)
        par = codec.encode([bytes(d) for d in data])
        assert sha(b"".join(par)) == c["parity_sha256"]


def test_device_batch_full_size(ctx):
    """Bench workload (k=128 batch) on device-resident buffers: sampled squares
    bit-exact vs the oracle, all squares vs the host API, and the Q3 identity
    (column-extension of Q1 == row-extension of Q2) on every square."""
    import torch
    from celestia_da.device import DeviceSquares

    k, n = 128, 16
    ds = DeviceSquares(k, n, ctx=ctx)
    host = np.stack([synth.random_blob_square(k, 7000 + i).reshape(-1) for i in range(n)])
    ds.ods.copy_(torch.from_numpy(host))
    ds.extend()
    torch.cuda.synchronize()
    dah = ds.dah.cpu().numpy()
    assert (ds.status.cpu().numpy() == 0).all()
    assert len({d.tobytes() for d in dah}) == n
    for i in (0, n - 1):
        _, orr, ocr, odah = oracle.extend_and_dah(host[i], k, nthreads=8, want_eds=False)
        assert dah[i].tobytes() == odah
        assert (ds.row_roots[i].cpu().numpy() == orr).all()
    _, _, _, hdah, st = da.extend_batch(host.reshape(-1), [k] * n, ctx)
    assert (hdah == dah).all()
    # Q3 identity on the device EDS for every square
    eds = ds.eds.view(n, 2 * k, 2 * k, 512).cpu().numpy()
    codec = da.LeoRSCodec(ctx)
    q1cols = np.ascontiguousarray(eds[:, :k, k:, :].transpose(0, 2, 1, 3)).reshape(n * k, k, 512)
    q3cols = np.ascontiguousarray(eds[:, k:, k:, :].transpose(0, 2, 1, 3)).reshape(n * k, k, 512)
    assert (codec.encode_batch(q1cols) == q3cols).all()
    # rerun is deterministic
    ds.extend()
    torch.cuda.synchronize()
    assert (ds.dah.cpu().numpy() == dah).all()


# --- decode / Repair (rsmt2d Repair, klauspost Reconstruct) -------------------

@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128])
@pytest.mark.parametrize("shard", [64, 512, 1536])
def test_codec_decode_matches_oracle(ctx, k, shard):
    rng = np.random.default_rng(k * 7 + shard)
    codec = da.LeoRSCodec(ctx)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    for trial in range(3):
        keep = rng.choice(2 * k, k + trial * (k // 4), replace=False)
        shards = [full[i].tobytes() if i in set(keep.tolist()) else None for i in range(2 * k)]
        out = codec.decode(shards)
        assert b"".join(out) == full.tobytes()


@pytest.mark.parametrize("pattern", ["data_half", "parity_half", "alternate", "first_k_plus_1"])
def test_codec_decode_k128_structured(ctx, pattern):
    """The bit-sliced k = 128 decoder (rs_decode_sliced.hip, whole 512-B chunks;
    4 chunks here) on structured erasures: every data shard lost, every parity
    shard lost, every other shard lost, and k + 1 present at the front."""
    k, shard = 128, 2048
    rng = np.random.default_rng(31 * len(pattern))
    codec = da.LeoRSCodec(ctx)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    idx = np.arange(2 * k)
    keep = {"data_half": idx >= k, "parity_half": idx < k, "alternate": idx % 2 == 0,
            "first_k_plus_1": idx <= k}[pattern]
    shards = [full[i].tobytes() if keep[i] else None for i in range(2 * k)]
    out = codec.decode(shards)
    assert b"".join(out) == full.tobytes()


@pytest.mark.parametrize("nvec,k,shard", [(300, 16, 512), (1100, 4, 64), (24, 128, 512)])
def test_codec_decode_batch_shared_patterns(ctx, nvec, k, shard):
    """dagpu_decode over many vectors in one call: runs of equal erasure
    patterns share their error locators (one workgroup scans <= 1024 vectors;
    larger batches decode without sharing), mixed with distinct patterns."""
    from celestia_da import _abi
    rng = np.random.default_rng(nvec + k)
    data = rng.integers(0, 256, (nvec, k, shard), dtype=np.uint8)
    full = np.stack([np.concatenate([d, oracle.encode(d)]) for d in data])
    present = np.zeros((nvec, 2 * k), np.uint8)
    v = 0
    while v < nvec:
        run = int(rng.integers(1, 6))
        pat = np.zeros(2 * k, np.uint8)
        pat[rng.choice(2 * k, k + int(rng.integers(0, k + 1)) if k > 1 else 1, replace=False)] = 1
        present[v:v + run] = pat
        v += run
    buf = (full * present[:, :, None]).copy()
    ctx.check(ctx._L.dagpu_decode(ctx.handle, k, nvec, shard, _abi.addr(buf), _abi.addr(present)))
    assert np.array_equal(buf, full)


def test_codec_decode_too_few(ctx):
    k = 8
    codec = da.LeoRSCodec(ctx)
    shards = [bytes(64)] * (k - 1) + [None] * (k + 1)
    with pytest.raises(da.ErrTooFewShards):
        codec.decode(shards)


def _subgrid(k, seed):
    rng = np.random.default_rng(seed)
    w = 2 * k
    present = np.zeros((w, w), bool)
    present[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
    return present


@pytest.mark.parametrize("k", [1, 2, 8, 32, 128])
def test_repair_max_erasure(ctx, k):
    """C4: keep a k x k sub-grid (3k^2 erased), repair, every root re-verified."""
    ods = synth.random_blob_square(k, 40 + k)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k, nthreads=8)
    present = _subgrid(k, k)
    damaged = eds * present[:, :, None]
    fixed, pres = da.repair(damaged, present, rr, cr, ctx)
    assert pres.all()
    assert (fixed == eds).all()


@pytest.mark.parametrize("k", [1, 2, 8, 32, 128])
def test_repair_q3_only_host_api(ctx, k):
    """C4 with the other maximal pattern, Q3 only kept (the reverse fill's
    case: every kept row and column has a complete parity half), through the
    single-square host entry point (dagpu_repair), against the oracle's repair."""
    ods = synth.random_blob_square(k, 70 + k)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k, nthreads=8)
    w = 2 * k
    present = np.zeros((w, w), bool)
    present[k:, k:] = True
    damaged = eds * present[:, :, None]
    fixed, pres = da.repair(damaged, present, rr, cr, ctx)
    assert pres.all() and (fixed == eds).all()
    if k <= 32:
        orc, ofixed = oracle.repair(damaged, present, k, rr, cr)
        assert orc == 0 and (ofixed == fixed).all()


@pytest.mark.parametrize("k", [4, 16])
def test_repair_random_patterns_match_oracle(ctx, k):
    rng = np.random.default_rng(k)
    ods = synth.random_blob_square(k, 60 + k)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k)
    w = 2 * k
    for frac in (0.3, 0.45, 0.6, 0.9):
        present = rng.random((w, w)) < frac
        damaged = eds * present[:, :, None]
        orc, ofixed = oracle.repair(damaged, present, k, rr, cr)
        try:
            fixed, _ = da.repair(damaged, present, rr, cr, ctx)
            code = 0
        except da.DAError as e:
            code, fixed = e.code, None
        assert code == orc, frac
        if code == 0:
            assert (fixed == ofixed).all() and (fixed == eds).all()


def test_repair_byzantine_and_errors(ctx):
    k = 8
    w = 2 * k
    ods = synth.random_blob_square(k, 99)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k)
    present = _subgrid(k, 1)
    damaged = eds * present[:, :, None]
    # corrupt one present share: the rebuilt axes no longer match the roots
    r, c = np.argwhere(present)[0]
    bad = damaged.copy()
    bad[r, c, 200] ^= 0x40
    with pytest.raises(da.ErrByzantineData):
        da.repair(bad, present, rr, cr, ctx)
    # too few shares everywhere -> unrepairable
    few = present.copy()
    few[r, :] = False
    few[:, c] = False
    with pytest.raises(da.ErrUnrepairableDataSquare):
        da.repair(eds * few[:, :, None], few, rr, cr, ctx)
    # complete square whose parity is inconsistent but roots commit to it:
    # prerepairSanityCheck -> ErrByzantineData
    inc = eds.copy()
    inc[0, w - 1, 7] ^= 1
    irr, icr = oracle.compute_roots(inc, k)
    full = np.ones((w, w), bool)
    full[w - 1, w - 1] = False
    with pytest.raises(da.ErrByzantineData):
        da.repair(inc, full, irr, icr, ctx)
    # complete axis with a wrong root -> "bad root input"
    wrong = rr.copy()
    wrong[0, 70] ^= 1
    with pytest.raises(da.DAError, match="bad root input"):
        da.repair(eds, full, wrong, cr, ctx)
    # nothing missing and consistent -> no-op
    fixed, _ = da.repair(eds, np.ones((w, w), bool), rr, cr, ctx)
    assert (fixed == eds).all()


def test_repair_k128_byzantine_and_unrepairable(ctx):
    """The error classes through the bit-sliced k = 128 decoder: a corrupted
    present share under the maximal erasure pattern makes the rebuilt axes
    miss their roots (ErrByzantineData); one row and one column fewer leaves
    nothing decodable (ErrUnrepairableDataSquare)."""
    k = 128
    w = 2 * k
    ods = synth.random_blob_square(k, 4242)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k, nthreads=8)
    present = _subgrid(k, 77)
    r, c = np.argwhere(present)[5]
    bad = eds * present[:, :, None]
    bad[r, c, 311] ^= 0x08
    with pytest.raises(da.ErrByzantineData):
        da.repair(bad, present, rr, cr, ctx)
    few = present.copy()
    few[r, :] = False
    few[:, c] = False
    with pytest.raises(da.ErrUnrepairableDataSquare):
        da.repair(eds * few[:, :, None], few, rr, cr, ctx)


def test_repair_device_batch(ctx):
    """C4 on the device-resident batch API: 8 squares at k=128."""
    import torch
    from celestia_da.device import DeviceSquares

    k, n = 128, 8
    ds = DeviceSquares(k, n, ctx=ctx)
    host = np.stack([synth.random_blob_square(k, 8100 + i).reshape(-1) for i in range(n)])
    ds.ods.copy_(torch.from_numpy(host))
    ds.extend()
    eds_ref = ds.eds.clone()
    w = 2 * k
    pres = np.stack([_subgrid(k, 500 + i).reshape(-1) for i in range(n)]).astype(np.uint8)
    present = torch.from_numpy(pres).cuda()
    mask = present.view(n, w * w, 1).to(torch.uint8)
    ds.eds.copy_((ds.eds.view(n, w * w, 512) * mask).view(n, -1))
    status = torch.full((n,), -99, dtype=torch.int32, device="cuda")
    ws = ds.repair_workspace()
    ds.repair(present, status, ws)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert bool((present == 1).all())
    assert torch.equal(ds.eds, eds_ref)


def test_repair_device_batch_mixed_outcomes(ctx):
    """C4 on a 64-square device batch at k = 64: distinct maximal erasure
    patterns, one byzantine square and one unrepairable square; every status
    lands on its own square and every other square is rebuilt bit-exactly."""
    import torch
    from celestia_da.device import DeviceSquares

    k, n = 64, 64
    w = 2 * k
    ds = DeviceSquares(k, n, ctx=ctx)
    host = synth.blob_squares(k, 6464, 0, n)
    ds.load_ods(host)
    ds.extend()
    eds_ref = ds.eds.clone()
    pres = np.stack([_subgrid(k, 900 + i) for i in range(n)])
    byz, unrep = 20, 40
    r, c = np.argwhere(pres[unrep])[0]
    pres[unrep][r, :] = False
    pres[unrep][:, c] = False
    present = torch.from_numpy(pres.reshape(n, -1).astype(np.uint8)).cuda()
    mask = present.view(n, w * w, 1)
    ds.eds.copy_((ds.eds.view(n, w * w, 512) * mask).view(n, -1))
    rb, cb = np.argwhere(pres[byz])[3]
    ds.eds.view(n, w, w, 512)[byz, rb, cb, 77] ^= 0x10
    status = torch.full((n,), -99, dtype=torch.int32, device="cuda")
    ds.repair(present, status, ds.repair_workspace())
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    want = np.zeros(n, np.int32)
    want[byz], want[unrep] = _abi.ERR_BYZANTINE, _abi.ERR_UNREPAIRABLE
    assert (st == want).all(), st
    ok = [i for i in range(n) if i not in (byz, unrep)]
    assert torch.equal(ds.eds[ok], eds_ref[ok])
    assert bool((present[ok] == 1).all())
