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


def _prototypes(header):
    """{name: argument count} of every nicgpu_* prototype in the header."""
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"//[^\n]*", "", text)
    out = {}
    for name, args in re.findall(r"(?:int|const char\*)\s+(nicgpu_\w+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        args = args.strip()
        out[name] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_signatures_match_header_prototypes():
    """Every ctypes signature the package binds has the header's argument
    count (nicgpu_qp_verify_fixups_async was bound with three)."""
    protos = _prototypes("nicgpu.h")
    sigs = sna.signatures()
    assert set(sigs) <= set(protos), sorted(set(sigs) - set(protos))
    bad = {n: (len(a), protos[n]) for n, (_, a) in sigs.items() if len(a) != protos[n]}
    assert not bad, bad
    assert len(sigs) >= 60  # (nearly every entry point is bound)


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
    assert lib.nicgpu_abi_version() == 2 == sna.ABI_VERSION
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


def test_batch_entry_points_validate_before_device_access():
    """Every batch entry point of include/nicgpu.h checks its arguments before
    touching a device (so the results below hold with or without a GPU): an
    empty batch is a no-op, missing buffers, a misaligned frame base, a bad
    ICRC mode or a zero slot stride are NICGPU_ERR_INVALID."""
    lib = sna.load_library()
    buf = (ctypes.c_uint8 * 64)()
    base = ctypes.addressof(buf)
    aligned = (base + 15) & ~15
    mis = aligned + 1
    p = aligned  # any non-null pointer for the other arguments
    OK, INV = sna.OK, sna.ERR_INVALID
    # nicgpu_tso_checksum(frames, desc, hdr_len, mss, seg_base, n, out, stream)
    assert lib.nicgpu_tso_checksum(None, None, None, None, None, 0, None, None) == OK
    assert lib.nicgpu_tso_checksum(None, p, p, p, p, 1, p, None) == INV
    assert lib.nicgpu_tso_checksum(p, p, p, p, p, 1, None, None) == INV
    assert lib.nicgpu_tso_checksum(mis, p, p, p, p, 1, p, None) == INV
    # nicgpu_tso_segment(frames, desc, hdr, mss, seg_base, flags, n, out, out_size, stride, out_len, out_csum, stream)
    assert lib.nicgpu_tso_segment(None, None, None, None, None, None, 0, None, 0, 0, None, None, None) == OK
    assert lib.nicgpu_tso_segment(p, p, p, p, p, None, 1, None, 64, 16, None, None, None) == INV
    assert lib.nicgpu_tso_segment(p, p, p, p, p, None, 1, p, 64, 0, None, None, None) == INV
    assert lib.nicgpu_tso_segment(mis, p, p, p, p, None, 1, p, 64, 16, None, None, None) == INV
    # nicgpu_icrc_batch(frames, desc, n, mode, out_crc, out_ok, stream)
    assert lib.nicgpu_icrc_batch(p, p, 1, 2, p, None, None) == INV            # unknown mode
    assert lib.nicgpu_icrc_batch(p, p, 1, 0, p, p, None) == INV               # CALCULATE with out_ok
    assert lib.nicgpu_icrc_batch(p, p, 1, 1, p, None, None) == INV            # VERIFY without out_ok
    assert lib.nicgpu_icrc_batch(None, None, 0, 0, None, None, None) == OK
    assert lib.nicgpu_icrc_batch(None, p, 1, 0, p, None, None) == INV
    assert lib.nicgpu_icrc_batch(mis, p, 1, 0, p, None, None) == INV
    # nicgpu_segment_gather(mem, mem_size, writes, n, stream)
    assert lib.nicgpu_segment_gather(None, 0, None, 0, None) == OK
    assert lib.nicgpu_segment_gather(None, 64, p, 1, None) == INV
    assert lib.nicgpu_segment_gather(p, 64, None, 1, None) == INV
    # nicgpu_segment_gather_from(mem, src, mem_size, writes, n, stream)
    assert lib.nicgpu_segment_gather_from(None, None, 0, None, 0, None) == OK
    assert lib.nicgpu_segment_gather_from(None, p, 64, p, 1, None) == INV
    assert lib.nicgpu_segment_gather_from(p, None, 64, p, 1, None) == INV
    assert lib.nicgpu_segment_gather_from(p, p, 64, None, 1, None) == INV
    # nicgpu_checksum_batch(frames, desc, n, out, stream): the RX pass without RSS
    assert lib.nicgpu_checksum_batch(None, None, 0, None, None) == OK
    assert lib.nicgpu_checksum_batch(None, p, 1, p, None) == INV
    assert lib.nicgpu_checksum_batch(p, None, 1, p, None) == INV
    assert lib.nicgpu_checksum_batch(mis, p, 1, p, None) == INV
    # the device QueuePair context (nicgpu_qp_*): no context, no outputs -> INVALID
    assert lib.nicgpu_qp_create(None, 0) == INV
    assert lib.nicgpu_qp_destroy(None) == INV
    assert lib.nicgpu_qp_reserve(None, 1, 1, p) == INV
    assert lib.nicgpu_qp_plan(None, p, 64, 1, 9000, p, p, None) == INV
    assert lib.nicgpu_qp_plan_on(None, p, 64, 1, 9000, p, p, None, None) == INV
    # streams and events: null handles -> INVALID (no device touched)
    assert lib.nicgpu_stream_create(None) == INV
    assert lib.nicgpu_stream_destroy(None) == INV
    assert lib.nicgpu_event_create(None) == INV
    assert lib.nicgpu_event_destroy(None) == INV
    assert lib.nicgpu_event_record(None, None) == INV
    assert lib.nicgpu_stream_wait_event(None, None) == INV
    assert lib.nicgpu_qp_check(None, 64, 1, 1, p, None) == INV
    assert lib.nicgpu_qp_resolve(None, 64, 1, 1, 9000, 0, p, p, p, None) == INV
    assert lib.nicgpu_qp_rss_list(None, 1, None) == INV
    assert lib.nicgpu_qp_rss_scatter(None, 1, None) == INV
    assert lib.nicgpu_qp_group(None, 1, 4, None) == INV
    # nicgpu_rx_offload_ex(ctx, frames, desc, n, mode, raw_off, raw_len, csum, hash, queue, hits, l34, stream)
    NONE, AUTO, RAW = sna.TUPLE_NONE, sna.TUPLE_AUTO, sna.TUPLE_RAW
    # nicgpu_rx_offload_count: a device count is required; then the same checks as nicgpu_rx_offload
    assert lib.nicgpu_rx_offload_count(None, p, p, 1, None, NONE, 0, 0, p, None, None, None, None) == INV
    assert lib.nicgpu_rx_offload_count(None, mis, p, 1, p, NONE, 0, 0, p, None, None, None, None) == INV
    assert lib.nicgpu_rx_offload_count(None, p, p, 1, p, AUTO, 0, 0, p, p, p, None, None) == INV  # RSS without ctx
    assert lib.nicgpu_rx_offload_ex(None, None, None, 0, NONE, 0, 0, None, None, None, None, None, None) == OK
    assert lib.nicgpu_rx_offload_ex(None, None, p, 1, NONE, 0, 0, p, None, None, None, p, None) == INV
    assert lib.nicgpu_rx_offload_ex(None, p, None, 1, NONE, 0, 0, p, None, None, None, p, None) == INV
    assert lib.nicgpu_rx_offload_ex(None, mis, p, 1, NONE, 0, 0, p, None, None, None, p, None) == INV
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, NONE, 0, 0, None, p, None, None, None, None) == INV  # hash without RSS
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, NONE, 0, 0, None, None, p, None, None, None) == INV  # queue without RSS
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, NONE, 0, 0, None, None, None, p, None, None) == INV  # hits without RSS
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, 7, 0, 0, p, None, None, None, None, None) == INV     # unknown mode
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, RAW, 60, 8, p, None, None, None, None, None) == INV  # window past 64 B
    assert lib.nicgpu_rx_offload_ex(None, p, p, 1, AUTO, 0, 0, p, p, p, None, None, None) == INV      # RSS without ctx
