"""The Repair reverse fill's identity on the CPU (oracle/pyref.py, pure Python):
Leopard's encode is parity = FFT(skew offset 0) of IFFT(skew offset m) of the
data, both over one polynomial of degree < m (klauspost/reedsolomon
leopard8.go encode: ifftDITEncoder8 with fftSkew[m-1:], then fftDIT8 with
fftSkew), so FFT(offset m) of IFFT(offset 0) of the parity is the data again.
The GPU kernels (EncodeArgs.reverse in rs_gf8.hip, rs_gf8_sliced.hip,
rs_gf16.hip) compute exactly this with the skew offsets swapped; the GF(2^8)
case is checked here for every power-of-two m, the GPU paths against the
oracle's decoder in tests/test_gpu_repair_fill.py."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import pyref as P  # noqa: E402


def _transform(data, io, fo):
    """ifftDIT8 at skew offset io, then fftDIT8 at skew offset fo (m = len(data))."""
    m = len(data)
    w = [bytearray(d) for d in data]
    dist, dist4 = 1, 4
    while dist4 <= m:
        for r in range(0, m, dist4):
            iend = r + dist
            l01, l02, l23 = (P.SKEW[io - 1 + iend], P.SKEW[io - 1 + iend + dist],
                             P.SKEW[io - 1 + iend + 2 * dist])
            for i in range(r, iend):
                P._ifft2(w, i, i + dist, l01)
                P._ifft2(w, i + 2 * dist, i + 3 * dist, l23)
                P._ifft2(w, i, i + 2 * dist, l02)
                P._ifft2(w, i + dist, i + 3 * dist, l02)
        dist, dist4 = dist4, dist4 << 2
    if dist < m:
        for i in range(dist):
            P._ifft2(w, i, i + dist, P.SKEW[io - 1 + dist])
    dist4, dist = m, m >> 2
    while dist:
        for r in range(0, m, dist4):
            iend = r + dist
            l01, l02, l23 = (P.SKEW[fo + iend - 1], P.SKEW[fo + iend + dist - 1],
                             P.SKEW[fo + iend + 2 * dist - 1])
            for i in range(r, iend):
                P._fft2(w, i, i + 2 * dist, l02)
                P._fft2(w, i + dist, i + 3 * dist, l02)
                P._fft2(w, i, i + dist, l01)
                P._fft2(w, i + 2 * dist, i + 3 * dist, l23)
        dist4, dist = dist, dist >> 2
    if dist4 == 2:
        for r in range(0, m, 2):
            P._fft2(w, r, r + 1, P.SKEW[fo + r])
    return [bytes(x) for x in w]


@pytest.mark.parametrize("m", [1, 2, 4, 8, 16, 32, 64, 128])
def test_reverse_transform_inverts_encode(m):
    rng = random.Random(31 + m)
    for _ in range(2):
        data = [bytes(rng.randrange(256) for _ in range(8)) for _ in range(m)]
        parity = P.encode(data)
        assert _transform(data, m, 0) == parity  # the forward form is the encoder
        assert _transform(parity, 0, m) == data
