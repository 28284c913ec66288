"""The k = 16384 split square (include/dagpu.h DAGPU_MAX_SPLIT_WIDTH): a
512 GiB EDS, which only the P >= 8 split path serves
(pkg/da/data_availability_header.go:65-75 ExtendShares puts no upper bound on
k; rsmt2d's Leopard codec serves it).  The whole square needs eight GPUs, so
this single-GPU test checks ONE part of a P = 64 split end to end and the
finish step on its own:

  * all 64 row owners' step 1 run here one after another (each on its 256 Q0
    rows, 2 GiB of seeded synthetic shares), and their send blocks for part g
    assemble g's slab exactly as the all-to-all would;
  * part g (a Q1 column slab) runs step 3: sampled slab rows against the
    oracle's row encoder, sampled columns against its column encoder and
    wrapper tree (column roots), sampled row-subtree records against its NMT;
  * step 5 on synthetic subtree records and column roots: sampled row roots
    against the oracle's NMT over the P records, the DAH against its RFC-6962.

Parity unpinned (GF(2^16): no reference vector at this width); oracle =
oracle/da_oracle.c.  Unmeasured on hardware as a whole square: the eight-GPU
run is the driver's node, not this box."""
import numpy as np
import pytest
import torch

import oracle
from celestia_da import _abi, da
from celestia_da.split import REC, SplitPart

pytestmark = pytest.mark.gpu

K = 16384
P = 64
NS_Q0 = bytes([0] * 19 + [7] * 10)
PARITY_NS = b"\xff" * 29


@pytest.fixture(scope="module")
def ctx():
    c = da.Context(0)
    yield c
    c.close()


def _rows_chunk(h: int, rows: int) -> torch.Tensor:
    """Q0 rows [h*rows, (h+1)*rows): seeded random shares, one namespace (sorted)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(1000 + h)
    t = torch.randint(0, 256, (rows, K, 512), dtype=torch.uint8, device="cuda", generator=g)
    t[:, :, :29] = torch.frombuffer(bytearray(NS_Q0), dtype=torch.uint8).cuda()
    return t


def _root(cells: np.ndarray, keep_ns: bool) -> bytes:
    leaves = [oracle.nmt_leaf(bytes(c[:29]) if keep_ns else PARITY_NS, c.tobytes()) for c in cells]
    return oracle.nmt_root(leaves)


def _rec_to_node(rec: bytes) -> bytes:
    return rec[0:29] + rec[32:61] + rec[64:96]


def test_split_k16384_limits(ctx):
    L = ctx._L
    assert L.dagpu_split_workspace_size(K, 4) == 0  # a 512 GiB EDS over 4 GPUs does not fit
    assert L.dagpu_split_workspace_size(K, 8) > 0
    assert L.dagpu_split_workspace_size(2 * K, 64) == 0
    with pytest.raises(da.DAError, match="needs >= 8 parts"):
        SplitPart(K, 4, 0, ctx, torch.device("cuda"))


def test_split_k16384_one_part_of_64(ctx):
    dev = torch.device("cuda")
    w = 2 * K
    g = P // 2 + 3  # a Q1 column slab: its top half is row parity
    mine = SplitPart(K, P, g, ctx, dev)
    owner = SplitPart(K, P, 0, ctx, dev)  # every row owner's step 1, one after another
    rows, W = mine.rows, mine.W
    blk = rows * W * 512
    rng = np.random.default_rng(16384)
    sample_rows = sorted(rng.choice(K, 2, replace=False).tolist())
    kept = {}
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    for h in range(P):
        chunk = _rows_chunk(h, rows)
        owner.step_rows(chunk.view(-1))
        status = torch.maximum(status, owner.status)
        mine.slab_top[h * blk:(h + 1) * blk].copy_(owner.send[g * blk:(g + 1) * blk])
        for r in sample_rows:
            if h * rows <= r < (h + 1) * rows:
                kept[r] = chunk[r - h * rows].cpu().numpy()
        del chunk
    mine.step_cols()
    torch.cuda.synchronize()
    assert int(status.item()) == 0 and int(mine.status.item()) == 0
    print("k=16384 part: rows and columns stepped", flush=True)
    slab = mine.slab.view(w, W, 512)
    c0 = g * W - K  # first parity column of the slab
    for r, row in kept.items():  # slab rows 0..k-1 = the rows' parity at the slab's columns
        assert (slab[r].cpu().numpy() == oracle.encode(row)[c0:c0 + W]).all(), r
    col_roots = mine.col_roots.view(W, 90).cpu().numpy()
    for c in (0, W - 1):
        col = slab[:, c].cpu().numpy()
        assert (col[K:] == oracle.encode(np.ascontiguousarray(col[:K]))).all(), c
        assert col_roots[c].tobytes() == _root(col, False), c  # column g*W + c >= k: parity namespaces
    row_sub = mine.row_sub.view(w, REC).cpu().numpy()
    for r in (3, K - 1, K + 11, w - 1):
        want = _root(slab[r].cpu().numpy(), False)
        assert _rec_to_node(row_sub[r].tobytes()) == want, r
    print("k=16384 part: sampled rows, columns, roots and subtrees checked", flush=True)
    del owner
    torch.cuda.empty_cache()

    # step 5 at k = 16384 on synthetic inputs: part p's record of row r keeps
    # the Q0 namespace where the row's cells under p are Q0 (r < k, p < P/2)
    recs = np.zeros((P, w, REC), np.uint8)
    recs[:, :, 64:] = rng.integers(0, 256, (P, w, 32), dtype=np.uint8)
    ns = np.frombuffer(PARITY_NS, np.uint8)
    recs[:, :, 0:29] = ns
    recs[:, :, 32:61] = ns
    q0 = np.frombuffer(NS_Q0, np.uint8)
    recs[:P // 2, :K, 0:29] = q0
    recs[:P // 2, :K, 32:61] = q0
    cols = np.zeros((w, 90), np.uint8)
    cols[:, :58] = np.concatenate([ns, ns])
    cols[:K, :29] = q0
    cols[:, 58:] = rng.integers(0, 256, (w, 32), dtype=np.uint8)
    rr, dah = mine.step_finish(torch.from_numpy(recs.reshape(-1)).to(dev), torch.from_numpy(cols.reshape(-1)).to(dev))
    torch.cuda.synchronize()
    rr = rr.view(w, 90).cpu().numpy()
    for r in (0, K - 1, K, w - 1):
        want = oracle.nmt_root([_rec_to_node(recs[p, r].tobytes()) for p in range(P)])
        assert rr[r].tobytes() == want, r
    assert bytes(dah.cpu().numpy()) == oracle.dah_hash(rr, cols)
    del mine
    torch.cuda.empty_cache()
