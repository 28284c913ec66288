"""CPU tests of the C-ABI library: it loads, exports every symbol the header
declares, fails cleanly without a GPU, and its host-side helpers agree with
the oracle.  No GPU compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import oracle
from celestia_da import _abi, da, synth

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dagpu.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dagpu_[a-z_0-9]+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    L = _abi.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_abi.EXPORTS)
    assert L.dagpu_version() >= 100


def test_library_is_gfx950_code_object():
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only check")
def test_init_without_gpu_fails_cleanly():
    h = ctypes.c_void_p()
    rc = _abi.lib().dagpu_init(0, ctypes.byref(h))
    assert rc in (_abi.ERR_DEVICE, _abi.ERR_ARG)
    assert not h.value


def test_dah_hash_host_helper_matches_oracle():
    # nil DAH (pkg/da/data_availability_header_test.go:15-25)
    assert da.nil_dah_hash().hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    for k in (1, 2, 8):
        ods = synth.random_blob_square(k, 11 * k)
        _, rr, cr, dah = oracle.extend_and_dah(ods, k)
        h = da.DataAvailabilityHeader([bytes(r) for r in rr], [bytes(c) for c in cr])
        assert h.hash() == dah
        h.validate_basic()
        assert h.square_size() == k


def test_validation_errors_before_device():
    # pkg/da/data_availability_header_test.go:70-99
    with pytest.raises(da.DAError, match="number of shares is not a power of 2: got 5"):
        da.extend_shares([b"\x00" * 512] * 5)
    with pytest.raises(da.DAError, match="not a power of 2"):
        da.extend_shares([b"\x00" * 512] * (129 * 129))
    with pytest.raises(da.DAError, match="square number"):
        da.extend_shares([b"\x00" * 512] * 8)
    with pytest.raises(da.DAError):
        da.extend_shares([b"\x00" * 512] * 0)


def test_validate_basic_bounds():
    r = b"\x00" * 90
    with pytest.raises(da.DAError, match="minimum valid"):
        da.DataAvailabilityHeader([r], [r]).validate_basic()
    with pytest.raises(da.DAError, match="maximum valid"):
        da.DataAvailabilityHeader([r] * 258, [r] * 258).validate_basic()
    with pytest.raises(da.DAError, match="unequal number"):
        da.DataAvailabilityHeader([r] * 4, [r] * 2).validate_basic()
    da.DataAvailabilityHeader([r] * 2, [r] * 2).validate_basic()


def test_square_size_helpers():
    # pkg/da/data_availability_header_test.go:217-243
    for n, want in [(0, 1), (1, 1), (2, 2), (4, 2), (5, 4), (16, 4), (17, 8), (16384, 128)]:
        assert da.square_size(n) == want, n
    assert da.is_power_of_two(1) and not da.is_power_of_two(0) and not da.is_power_of_two(6)


def test_min_shares_is_tail_padding():
    s = da.min_shares()
    assert len(s) == 1 and len(s[0]) == 512
    assert s[0][:29] == b"\xff" * 28 + b"\xfe" and s[0][29] == 1
    assert bytes(synth.tail_padding_square(1)[0]) == s[0]


def test_max_square_width_and_codec_limits():
    # the widest square the library serves: (2k)^2 x 512 B of EDS must fit one
    # GPU's 288 GB (k = 8192: 128 GiB; k = 16384: 512 GiB)
    L = _abi.lib()
    text = open(HEADER).read()
    m = re.search(r"#define DAGPU_MAX_SQUARE_WIDTH (\d+)", text)
    assert m and int(m.group(1)) == L.dagpu_max_square_width() == 8192
    m = re.search(r"#define DAGPU_MAX_CODEC_WIDTH (\d+)", text)
    assert m and int(m.group(1)) == L.dagpu_max_codec_width() == 32768  # Leopard: 65536 shards
    codec = da.LeoRSCodec()
    assert codec.max_chunks() == 32768 * 32768  # rsmt2d LeoRSCodec.MaxChunks
    assert codec.name() == "Leopard"


def test_codec_decode_without_any_shard_is_too_few():
    # reedsolomon Reconstruct with every shard nil -> ErrTooFewShards (no GPU
    # call is reached: the shard size cannot even be known)
    with pytest.raises(da.ErrTooFewShards):
        da.LeoRSCodec().decode([None] * 8)


def test_no_device_wait_on_later_queued_signals():
    # Invariant (DESIGN.md §4 "Started Repairs"): nothing on the device waits
    # for work queued later.  A stream wait on a signal word that a later
    # command releases hung once when two streams shared a hardware queue
    # (GPU_MAX_HW_QUEUES = 4); the library may only wait on events that are
    # already recorded.  Comments may name the primitive, code may not call it.
    csrc = os.path.join(ROOT, "celestia-app_amd", "csrc")
    bad = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".cpp", ".hip", ".hpp")):
            continue
        for no, line in enumerate(open(os.path.join(csrc, name)), 1):
            code = line.split("//", 1)[0]
            if re.search(r"hipStreamWait(Value|Write)|hipStreamWriteValue|hipStreamBatchMemOp", code):
                bad.append(f"{name}:{no}: {line.strip()}")
    assert not bad, bad


def test_split_widths_host_side():
    # k = 16384 (a 512 GiB EDS) only as a split square over >= 8 parts
    # (include/dagpu.h DAGPU_MAX_SPLIT_WIDTH); host-only sizing, no GPU call
    L = _abi.lib()
    text = open(HEADER).read()
    m = re.search(r"#define DAGPU_MAX_SPLIT_WIDTH (\d+)", text)
    assert m and int(m.group(1)) == 2 * L.dagpu_max_square_width() == 16384
    assert L.dagpu_split_workspace_size(8192, 1) > 0
    assert L.dagpu_split_workspace_size(16384, 4) == 0
    ws8 = L.dagpu_split_workspace_size(16384, 8)
    # per rank at P = 8: row staging 32 GiB + leaf / column / row forest records
    # ~38 GiB; with the 64 GiB slab and 32 GiB send block it stays under 288 GB
    assert 64 << 30 < ws8 < 80 << 30, ws8
    assert L.dagpu_split_workspace_size(16384, 64) > 0
    assert L.dagpu_split_workspace_size(32768, 64) == 0


def test_split_route_host_side():
    from celestia_da import split
    assert split.route(128, 1) == "single" and split.route(8192, 8) == "single"
    assert split.route(16384, 8) == "split" and split.route(16384, 64) == "split"
    for k, world in ((16384, 4), (16384, 1), (16384, 12), (32768, 64)):
        with pytest.raises(da.DAError) as e:
            split.route(k, world)
        assert e.value.code == _abi.ERR_UNSUPPORTED, (k, world)
    with pytest.raises(da.DAError):
        split.route(100, 8)
