"""The C ABI from a plain C program (tests/c_abi/dagpu_c_client.c, the calls a
cgo binding makes): golden DAH hashes of the reference
(pkg/da/data_availability_header_test.go), ExtendShares errors, the codec, the
page-locked batch API and one context per host thread."""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN

CLIENT = os.path.join(os.path.dirname(__file__), "c_abi", "dagpu_c_client")
REF = json.load(open(os.path.join(GOLDEN, "squares.json")))["reference"]


CLIENT_ASAN = CLIENT + "_asan"


def _run(client=CLIENT, env=None):
    assert os.path.exists(client), "build the client first: make -C celestia-app_amd c_client"
    p = subprocess.run([client], capture_output=True, text=True, timeout=300, env=env)
    return p.returncode, dict(line.split(" ", 1) for line in p.stdout.splitlines() if " " in line), p


def test_c_client_links_and_reports_device_errors_on_cpu():
    """Without a GPU the client still loads libdagpu.so and gets DAGPU_ERR_DEVICE."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    rc, out, p = _run()
    assert rc == 1 and out.get("init") == "-10", p.stdout + p.stderr


def _check_golden(rc, out, p):
    assert rc == 0, p.stdout + p.stderr
    assert out["init"] == "0" and p.stdout.strip().endswith("done")
    assert out["min_rc"] == "0" and out["min_dah"] == REF["min_dah"]["hash"]
    assert out["typical_rc"] == "0" and out["typical_dah"] == REF["typical_2x2"]["hash"]
    assert out["typical_q0_kept"] == "1"
    assert out["host_alloc"] == "1"
    assert out["max_rc"] == "0 0 0 0" and out["max_dah"] == REF["max_128x128"]["hash"]
    assert out["max_all_equal"] == "1"
    assert out["err_not_pow2"].split()[0] == "-1"
    assert "power of 2" in out["err_not_pow2"]
    assert out["err_not_square"] == "-2"
    assert out["err_push_order"] == "-4"
    assert out["codec_zero"] == "0 1"
    assert out["threads_ok"] == "1"
    assert out["pipelined"] == "-4 -4 1 1 -4"  # push-order status of square 21 only, same as unchunked


@pytest.mark.gpu
def test_c_client_golden_and_errors():
    _check_golden(*_run())


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(CLIENT_ASAN), reason="host-ASan build absent (make -C celestia-app_amd asan)")
def test_c_client_under_host_asan():
    """Same calls with the library's host code (plans, staging, pipelined
    batches, threads) built with AddressSanitizer; device code unchanged."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", DAGPU_CLIENT_QUICK_EXIT="1")
    rc, out, p = _run(CLIENT_ASAN, env)
    assert "ERROR: AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    _check_golden(rc, out, p)
