"""The GF(2^16) error-locator fold (csrc/rs_gf16.hip leo16_errlocs_fold_kernel)
on the CPU: for an erasure vector supported on [0, n), the first n outputs of
Leopard's 65536-point FWHT -> x logWalsh -> FWHT (leopard.go reconstruct,
restated in oracle/da_oracle.c) equal, mod 65535, two n-point transforms around
a multiply by the folded weights wfold[r] = sum_q logWalsh[q*n + r].  Checked
for n = 512 and 1024 on random and structured erasure patterns."""
import numpy as np
import pytest

import oracle

MOD = 65535


def fwht(v):
    """Walsh-Hadamard transform mod 65535 (any length 2^m), vectorised."""
    a = v.astype(np.int64) % MOD
    h = 1
    n = len(a)
    while h < n:
        a = a.reshape(-1, 2, h)
        s = (a[:, 0] + a[:, 1]) % MOD
        d = (a[:, 0] - a[:, 1]) % MOD
        a = np.stack([s, d], axis=1).reshape(n)
        h *= 2
    return a


@pytest.fixture(scope="module")
def log_walsh():
    log, _, _ = oracle.gf16_tables()
    w = log.astype(np.int64).copy()
    w[0] = 0
    return fwht(w)


@pytest.mark.parametrize("n", [512, 1024])
def test_fold_equals_full_transform(log_walsh, n):
    rng = np.random.default_rng(n)
    wfold = log_walsh.reshape(-1, n).sum(axis=0) % MOD
    patterns = [rng.random(n) < p for p in (0.1, 0.5, 0.9)]
    patterns.append(np.arange(n) < n // 2)        # every parity shard missing
    patterns.append(np.arange(n) % 3 == 0)
    for miss in patterns:
        e = np.zeros(65536, np.int64)
        e[:n] = miss
        full = fwht((fwht(e) * log_walsh) % MOD)[:n]
        fold = fwht((fwht(e[:n]) * wfold) % MOD)
        assert ((full - fold) % MOD == 0).all()
