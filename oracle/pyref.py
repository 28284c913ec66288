"""Pure-Python restatement of the DA hot path, for SMALL squares only (k <= 8).

TEST INFRASTRUCTURE ONLY.  An independent second restatement (python loops +
hashlib) used to cross-check the C oracle (da_oracle.c); same references:
  klauspost/reedsolomon v1.11.8 leopard8.go  (initLUTs8, initFFTSkew8,
      ifftDITEncoder8, fftDIT8)
  pkg/wrapper/nmt_wrapper.go:93-140, test/util/malicious/hasher.go:161-309
  celestia-core crypto/merkle HashFromByteSlices (RFC-6962)
"""
from __future__ import annotations

import hashlib
from typing import List

MOD = 255
CANTOR = [1, 214, 152, 146, 86, 200, 88, 230]
PARITY_NS = b"\xff" * 29


def _tables():
    exp = [0] * 256
    log = [0] * 256
    state = 1
    for i in range(MOD):
        exp[state] = i
        state <<= 1
        if state >= 256:
            state ^= 0x11D
    exp[0] = MOD
    log[0] = 0
    for i in range(8):
        width = 1 << i
        for j in range(width):
            log[j + width] = log[j] ^ CANTOR[i]
    log = [exp[v] for v in log]
    for i in range(256):
        exp[log[i]] = i
    exp[MOD] = exp[0]

    def add_mod(a, b):
        s = a + b
        return (s + (s >> 8)) & 0xFF

    def mullog(a, lb):
        return 0 if a == 0 else exp[add_mod(log[a], lb)]

    temp = [1 << i for i in range(1, 8)]
    skew = [0] * MOD
    for m in range(7):
        step = 1 << (m + 1)
        skew[(1 << m) - 1] = 0
        for i in range(m, 7):
            s = 1 << (i + 1)
            for j in range((1 << m) - 1, s, step):
                skew[j + s] = skew[j] ^ temp[i]
        temp[m] = MOD - log[mullog(temp[m], log[temp[m] ^ 1])]
        for i in range(m + 1, 7):
            temp[i] = mullog(temp[i], add_mod(log[temp[i] ^ 1], temp[m]))
    skew = [log[v] for v in skew]
    return log, exp, skew, mullog


LOG, EXP, SKEW, MULLOG = _tables()


def _xor(a: bytearray, b: bytes) -> None:
    for i in range(len(a)):
        a[i] ^= b[i]


def _muladd(x: bytearray, y: bytes, lm: int) -> None:
    lut = [MULLOG(v, lm) for v in range(256)]
    for i in range(len(x)):
        x[i] ^= lut[y[i]]


def _ifft2(w, i, j, lm):
    _xor(w[j], w[i])
    if lm != MOD:
        _muladd(w[i], w[j], lm)


def _fft2(w, i, j, lm):
    if lm != MOD:
        _muladd(w[i], w[j], lm)
    _xor(w[j], w[i])


def encode(data: List[bytes]) -> List[bytes]:
    """k data shards -> k parity shards (k power of two, 2k <= 256)."""
    m = len(data)
    w = [bytearray(d) for d in data]
    # ifftDITEncoder8, skewLUT = fftSkew[m-1:]
    dist, dist4 = 1, 4
    while dist4 <= m:
        for r in range(0, m, dist4):
            iend = r + dist
            l01, l02, l23 = SKEW[m - 1 + iend], SKEW[m - 1 + iend + dist], SKEW[m - 1 + iend + 2 * dist]
            for i in range(r, iend):
                _ifft2(w, i, i + dist, l01)
                _ifft2(w, i + 2 * dist, i + 3 * dist, l23)
                _ifft2(w, i, i + 2 * dist, l02)
                _ifft2(w, i + dist, i + 3 * dist, l02)
        dist, dist4 = dist4, dist4 << 2
    if dist < m:
        lm = SKEW[m - 1 + dist]
        for i in range(dist):
            _ifft2(w, i, i + dist, lm)
    # fftDIT8
    dist4, dist = m, m >> 2
    while dist:
        for r in range(0, m, dist4):
            iend = r + dist
            l01, l02, l23 = SKEW[iend - 1], SKEW[iend + dist - 1], SKEW[iend + 2 * dist - 1]
            for i in range(r, iend):
                _fft2(w, i, i + 2 * dist, l02)
                _fft2(w, i + dist, i + 3 * dist, l02)
                _fft2(w, i, i + dist, l01)
                _fft2(w, i + 2 * dist, i + 3 * dist, l23)
        dist4, dist = dist, dist >> 2
    if dist4 == 2:
        for r in range(0, m, 2):
            _fft2(w, r, r + 1, SKEW[r])
    return [bytes(x) for x in w]


def extend(ods: List[bytes], k: int) -> List[List[bytes]]:
    w = 2 * k
    eds = [[b""] * w for _ in range(w)]
    for r in range(k):
        for c in range(k):
            eds[r][c] = ods[r * k + c]
    for r in range(k):
        par = encode(eds[r][:k])
        for c in range(k):
            eds[r][k + c] = par[c]
    for c in range(k):
        par = encode([eds[r][c] for r in range(k)])
        for r in range(k):
            eds[k + r][c] = par[r]
    for r in range(k, w):
        par = encode(eds[r][:k])
        for c in range(k):
            eds[r][k + c] = par[c]
    return eds


def leaf(ns: bytes, data: bytes) -> bytes:
    return ns + ns + hashlib.sha256(b"\x00" + ns + data).digest()


def node(l: bytes, r: bytes) -> bytes:
    mx = l[29:58] if r[:29] == PARITY_NS else r[29:58]
    return l[:29] + mx + hashlib.sha256(b"\x01" + l + r).digest()


def nmt_root(leaves: List[bytes]) -> bytes:
    n = len(leaves)
    if n == 0:
        return b"\x00" * 58 + hashlib.sha256(b"").digest()
    if n == 1:
        return leaves[0]
    split = 1
    while split * 2 < n:
        split *= 2
    return node(nmt_root(leaves[:split]), nmt_root(leaves[split:]))


def axis_root(eds, k: int, axis: int, idx: int) -> bytes:
    w = 2 * k
    leaves = []
    for j in range(w):
        share = eds[idx][j] if axis == 0 else eds[j][idx]
        ns = share[:29] if (j < k and idx < k) else PARITY_NS
        leaves.append(leaf(ns, share))
    return nmt_root(leaves)


def rfc6962(items: List[bytes]) -> bytes:
    n = len(items)
    if n == 0:
        return hashlib.sha256(b"").digest()
    if n == 1:
        return hashlib.sha256(b"\x00" + items[0]).digest()
    split = 1
    while split * 2 < n:
        split *= 2
    return hashlib.sha256(b"\x01" + rfc6962(items[:split]) + rfc6962(items[split:])).digest()


def extend_and_dah(ods: List[bytes], k: int):
    eds = extend(ods, k)
    w = 2 * k
    rr = [axis_root(eds, k, 0, i) for i in range(w)]
    cr = [axis_root(eds, k, 1, i) for i in range(w)]
    return eds, rr, cr, rfc6962(rr + cr)


# ---- generic nmt / commitments (test oracle for dagpu_nmt_roots & co) -------------

def nmt_leaf_generic(namespaced_data: bytes) -> bytes:
    """nmt HashLeaf (test/util/malicious/hasher.go:186-209): ns | ns | H(0x00 | d)."""
    ns = namespaced_data[:29]
    return ns + ns + hashlib.sha256(b"\x00" + namespaced_data).digest()


def nmt_node_generic(l: bytes, r: bytes, ignore_max: bool) -> bytes:
    """nmt HashNode + computeNsRange (hasher.go:271-309)."""
    mx = l[29:58] if (ignore_max and r[:29] == PARITY_NS) else r[29:58]
    return l[:29] + mx + hashlib.sha256(b"\x01" + l + r).digest()


def nmt_root_generic(pushes: List[bytes], ignore_max: bool = True) -> bytes:
    """nmt computeRoot: RFC-6962 split at the largest power of two < n; empty
    tree = 0^29 | 0^29 | SHA256("") (hasher.go:161-168).  Raises ValueError on
    a push-order violation (nmt Push, ErrInvalidPushOrder)."""
    for a, b in zip(pushes, pushes[1:]):
        if b[:29] < a[:29]:
            raise ValueError("invalid push order")

    def rec(nodes):
        if len(nodes) == 0:
            return b"\x00" * 58 + hashlib.sha256(b"").digest()
        if len(nodes) == 1:
            return nodes[0]
        split = 1
        while split * 2 < len(nodes):
            split *= 2
        return nmt_node_generic(rec(nodes[:split]), rec(nodes[split:]), ignore_max)

    return rec([nmt_leaf_generic(p) for p in pushes])


def _round_up_pow2(v: int) -> int:
    r = 1
    while r < v:
        r <<= 1
    return r


def subtree_width(share_count: int, threshold: int = 64) -> int:
    """inclusion.SubTreeWidth (pkg/inclusion/blob_share_commitment_rules.go:85-101)
    with BlobMinSquareSize (:76-78)."""
    s = share_count // threshold + (1 if share_count % threshold else 0)
    s = _round_up_pow2(s)
    import math
    return min(s, _round_up_pow2(int(math.ceil(math.sqrt(share_count)))))


def mmr_sizes(total: int, max_tree: int) -> List[int]:
    """inclusion.MerkleMountainRangeSizes (pkg/inclusion/commitment.go:85-107)."""
    out = []
    while total:
        if total >= max_tree:
            t = max_tree
        else:
            up = _round_up_pow2(total)
            t = up if up == total else up // 2
        out.append(t)
        total -= t
    return out


def sparse_shares(ns: bytes, data: bytes, version: int = 0) -> List[bytes]:
    """SparseShareSplitter.Write for one blob (pkg/shares/split_sparse_shares.go:21-63,
    share_builder.go:56-80,155-221, info_byte.go:15-25)."""
    shares = []
    first = True
    while True:
        raw = bytearray(ns) + bytes([(version << 1) | (1 if first else 0)])
        if first:
            raw += len(data).to_bytes(4, "big")
        room = 512 - len(raw)
        raw += data[:room]
        data = data[room:]
        shares.append(bytes(raw) + b"\x00" * (512 - len(raw)))
        first = False
        if not data:
            return shares


def create_commitment(ns: bytes, data: bytes, threshold: int = 64, version: int = 0) -> bytes:
    """inclusion.CreateCommitment (pkg/inclusion/commitment.go:19-75)."""
    shares = sparse_shares(ns, data, version)
    sizes = mmr_sizes(len(shares), subtree_width(len(shares), threshold))
    roots, cur = [], 0
    for sz in sizes:
        roots.append(nmt_root_generic([ns + s for s in shares[cur:cur + sz]], True))
        cur += sz
    return rfc6962(roots)
