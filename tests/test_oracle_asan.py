"""The oracle (test infrastructure) under AddressSanitizer + UBSan: every
da_oracle.h entry point on small and edge-case inputs (oracle/asan_check.c)."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(__file__), "..", "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_clean_under_asan_ubsan():
    p = subprocess.run(["make", "-s", "-C", ORACLE, "asan"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "asan_check ok" in p.stdout
