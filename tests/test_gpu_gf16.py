"""GF(2^16) Leopard (2k > 256 shards: k = 256, 512) on the GPU.

klauspost/reedsolomon v1.11.8 switches to leopardFF16 when data + parity > 256
(leopard.go); rsmt2d reaches it for squares wider than 128.  No reference golden
vector covers this field (parity unpinned): the HIP kernels are compared
bit-for-bit with the oracle's GF(2^16) restatement, and erase -> decode round
trips must return the original bytes (an MDS decode is unique)."""
import numpy as np
import pytest

import oracle
from celestia_da import da, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("k", [256, 512])
@pytest.mark.parametrize("shard", [64, 320, 512, 1536])
def test_gf16_encode_matches_oracle(ctx, k, shard):
    rng = np.random.default_rng(k + shard)
    data = rng.integers(0, 256, (2, k, shard), dtype=np.uint8)
    par = da.LeoRSCodec(ctx).encode_batch(data)
    for v in range(2):
        assert (par[v] == oracle.encode(data[v])).all()


def test_gf16_encode_structured_inputs(ctx):
    # all-zero, all-0xFF and single-symbol inputs (log/exp edge entries 0 and 65535)
    k, shard = 256, 64
    codec = da.LeoRSCodec(ctx)
    cases = [np.zeros((k, shard), np.uint8), np.full((k, shard), 0xFF, np.uint8)]
    one = np.zeros((k, shard), np.uint8)
    one[3, 5] = 1
    one[3, 37] = 0x80  # high byte of symbol 5 in block 0
    cases.append(one)
    for data in cases:
        assert (codec.encode_batch(data[None])[0] == oracle.encode(data)).all()


@pytest.mark.parametrize("k", [256, 512])
def test_gf16_decode_round_trip(ctx, k):
    rng = np.random.default_rng(k * 3)
    codec = da.LeoRSCodec(ctx)
    shard = 128
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    for extra in (0, k // 3):
        keep = set(rng.choice(2 * k, k + extra, replace=False).tolist())
        shards = [full[i].tobytes() if i in keep else None for i in range(2 * k)]
        out = codec.decode(shards)
        assert b"".join(out) == full.tobytes()
    # only parity present / only data present
    for keep in (range(k, 2 * k), range(k)):
        keep = set(keep)
        shards = [full[i].tobytes() if i in keep else None for i in range(2 * k)]
        assert b"".join(codec.decode(shards)) == full.tobytes()


def test_gf16_decode_matches_oracle(ctx):
    k, shard = 256, 64
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    present = np.zeros(2 * k, np.uint8)
    present[rng.choice(2 * k, k + 7, replace=False)] = 1
    damaged = full * present[:, None]
    want = oracle.decode(damaged, present)
    got = da.LeoRSCodec(ctx).decode([damaged[i].tobytes() if present[i] else None for i in range(2 * k)])
    assert b"".join(got) == want.tobytes() == full.tobytes()


@pytest.mark.parametrize("shard", [256, 512, 1024])
def test_gf16_decode_k512_matches_oracle(ctx, shard):
    """k = 512 (n = 1024): shards that are whole 256-B pieces take the
    register-resident decoder (leo16_decode_reg1k_kernel); random erasure
    patterns with k .. 2k-1 survivors, only parity and only data present."""
    k = 512
    rng = np.random.default_rng(shard)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    codec = da.LeoRSCodec(ctx)
    pats = [np.isin(np.arange(2 * k), rng.choice(2 * k, k + extra, replace=False)) for extra in (0, 1, 100, k - 1)]
    pats += [np.arange(2 * k) >= k, np.arange(2 * k) < k]
    for present in pats:
        present = present.astype(np.uint8)
        damaged = full * present[:, None]
        if shard == 256:
            assert (oracle.decode(damaged, present) == full).all()
        got = codec.decode([damaged[i].tobytes() if present[i] else None for i in range(2 * k)])
        assert b"".join(got) == full.tobytes()


def test_gf16_decode_too_few(ctx):
    k = 256
    shards = [bytes(64)] * (k - 1) + [None] * (k + 1)
    with pytest.raises(da.ErrTooFewShards):
        da.LeoRSCodec(ctx).decode(shards)


@pytest.mark.parametrize("k", [256, 512])
def test_gf16_extend_matches_oracle(ctx, k):
    """C5 stress squares: EDS, every row/column root and the DAH hash."""
    ods = synth.random_blob_square(k, 900 + k)
    eds = da.extend_shares(ods, ctx)
    dah = da.new_data_availability_header(eds)
    oeds, orr, ocr, odah = oracle.extend_and_dah(ods, k, nthreads=8)
    assert (eds.data == oeds).all()
    assert b"".join(dah.row_roots) == orr.tobytes()
    assert b"".join(dah.column_roots) == ocr.tobytes()
    assert dah.hash() == odah
    # reference ValidateBasic caps the DAH at 256 roots per axis (k <= 128)
    with pytest.raises(da.DAError, match="maximum"):
        dah.validate_basic()


@pytest.mark.parametrize("k", [256, 512])
def test_gf16_repair_max_erasure(ctx, k):
    ods = synth.random_blob_square(k, 77)
    eds, rr, cr, _ = oracle.extend_and_dah(ods, k, nthreads=8)
    rng = np.random.default_rng(5)
    w = 2 * k
    present = np.zeros((w, w), bool)
    present[np.ix_(rng.choice(w, k, replace=False), rng.choice(w, k, replace=False))] = True
    fixed, pres = da.repair(eds * present[:, :, None], present, rr, cr, ctx)
    assert pres.all()
    assert (fixed == eds).all()
    # one corrupted surviving share -> byzantine
    bad = eds * present[:, :, None]
    r, c = np.argwhere(present)[0]
    bad[r, c, 100] ^= 1
    with pytest.raises(da.ErrByzantineData):
        da.repair(bad, present, rr, cr, ctx)


@pytest.mark.parametrize("k", [256, 512])
@pytest.mark.parametrize("shard", [64, 192, 256, 1536])
def test_halflane_encoders(ctx, k, shard):
    """The half-lane encoders (k = 512: two workgroups per CU, k = 256: four;
    256-B pieces, a partial last piece for 64 / 192 / 1536 B) against the oracle,
    for every vector of a batch."""
    rng = np.random.default_rng(3 * shard + k)
    data = rng.integers(0, 256, (3, k, shard), dtype=np.uint8)
    half = da.LeoRSCodec(ctx).encode_batch(data)
    for v in range(3):
        assert (half[v] == oracle.encode(data[v])).all(), v


@pytest.mark.parametrize("k", [512, 256])
@pytest.mark.parametrize("shard", [64, 192, 256, 768])
def test_gf16_decoders_all_shapes(ctx, k, shard):
    """The half-lane decoders (shards on the 256-B grid, missing shards not
    loaded) and the generic LDS decoder (64 / 192 B) rebuild the oracle's
    codewords under erasure patterns of every shape: random exactly-k, every
    other shard, a middle window, data half, parity half, over-determined."""
    rng = np.random.default_rng(29 + k + shard)
    data = rng.integers(0, 256, (k, shard), dtype=np.uint8)
    full = np.concatenate([data, oracle.encode(data)])
    codec = da.LeoRSCodec(ctx)
    for keep in (set(rng.choice(2 * k, k, replace=False).tolist()), set(range(0, 2 * k, 2)),
                 set(range(k // 2, k + k // 2)), set(range(k)), set(range(k, 2 * k)),
                 set(rng.choice(2 * k, k + 77, replace=False).tolist())):
        shards = [full[i].tobytes() if i in keep else None for i in range(2 * k)]
        assert b"".join(codec.decode(shards)) == full.tobytes()
