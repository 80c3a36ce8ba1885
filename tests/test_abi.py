"""The C-ABI library loads and exports every symbol include/nicgpu.h declares;
with no GPU it fails loudly (no CPU fallback).  CPU-only."""

import ctypes
import os
import re
import subprocess

import pytest

import smart_nic_amd as sna

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(nicgpu_\w+)\s*\(", text, re.M)))


def test_header_symbols_match_binding_list():
    assert _declared("nicgpu.h") == sorted(sna.ABI_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = sna.load_library()
    for name in _declared("nicgpu.h"):
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", sna.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (nicgpu_\w+)", out))
    assert set(_declared("nicgpu.h")) <= exported
    # tuning entry points never ship in the product library
    assert not any(s.startswith("nicgpu_tune") for s in exported)


def test_host_library_exports_nic_api():
    out = subprocess.run(["nm", "-DC", "--defined-only", sna.HOST_LIB_PATH], capture_output=True, text=True).stdout
    for sym in ["nic::compute_checksum(", "nic::verify_checksum(", "nic::compute_checksum_batch(",
                "nic::RssEngine::select_queue(", "nic::RssEngine::hash(", "nic::RssEngine::select_queue_batch(",
                "nic::RssEngine::set_key(", "nic::RssEngine::set_table(", "nic::RssEngine::reset_stats("]:
        assert sym in out, sym


def test_abi_version_and_errors_without_gpu():
    lib = sna.load_library()
    assert lib.nicgpu_abi_version() == 1
    assert lib.nicgpu_strerror(sna.ERR_NO_DEVICE) == b"no gfx950 device"
    # argument validation happens before any device access
    assert lib.nicgpu_rx_offload(None, None, None, 0, 7, 0, 0, None, None, None, None, None) == sna.ERR_INVALID
    assert lib.nicgpu_rx_offload(None, None, None, 4, sna.TUPLE_AUTO, 0, 0, None, None, None, None, None) == sna.ERR_INVALID
    # hashing without an RSS context is refused, never computed on the CPU
    assert lib.nicgpu_rx_offload(None, None, None, 4, sna.TUPLE_RAW, 60, 8, None, None, None, None, None) == sna.ERR_INVALID


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = sna.load_library()
    assert lib.nicgpu_device_count() <= 0
    h = ctypes.c_void_p()
    assert lib.nicgpu_rss_create(ctypes.byref(h), 0) == sna.ERR_NO_DEVICE
    buf = (ctypes.c_uint8 * 64)()
    desc = (ctypes.c_uint64 * 1)(16 << 40)
    out = (ctypes.c_uint16 * 1)()
    st = lib.nicgpu_checksum_batch(ctypes.addressof(buf) & ~15 or None, desc, 1, out, None)
    assert st in (sna.ERR_NO_DEVICE, sna.ERR_HIP, sna.ERR_INVALID)
