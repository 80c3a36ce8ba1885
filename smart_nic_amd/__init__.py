"""smart_nic_amd — MI355X-native RX offload path of smart_nic (checksum + RSS).

The product is native code: ``libnicgpu.so`` (HIP kernels for gfx950 behind the
C-ABI of ``include/nicgpu.h``) and ``libnic_host.so`` (the C++20 ``nic::`` API,
``include/nic/*.h``).  This Python package is glue for tests and ``bench.py``:
it binds the C-ABI with ctypes and passes torch-allocated device memory to it.
There is no CPU fallback — if the HIP library is missing or no gfx950 device
is visible every call raises.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NICGPU_LIB_AB: tools/ab_rows.sh points this at a side build for same-box A/B timing
LIB_PATH = os.environ.get("NICGPU_LIB_AB") or os.path.join(_HERE, "libnicgpu.so")
HOST_LIB_PATH = os.path.join(_HERE, "libnic_host.so")
INCLUDE_DIR = os.path.join(os.path.dirname(_HERE), "include")

# include/nicgpu.h
OK = 0
ERR_INVALID = -1
ERR_HIP = -2
ERR_NO_DEVICE = -3
ERR_NOMEM = -4
TUPLE_NONE = 0
TUPLE_AUTO = 1
TUPLE_RAW = 2
# L3/L4 verification flags (include/nicgpu.h NICGPU_L34_*)
L34_IPV4 = 0x01
L34_IPV4_OK = 0x02
L34_L4 = 0x04
L34_L4_OK = 0x08
L34_UDP_NOCSUM = 0x10
RAW_MAX_END = 64
MAX_PACKET = 65535
DESC_OFFSET_BITS = 40
ABI_VERSION = 2  # include/nicgpu.h NICGPU_ABI_VERSION

# Every symbol include/nicgpu.h declares (tests check the library exports them).
ABI_SYMBOLS = (
    "nicgpu_abi_version",
    "nicgpu_strerror",
    "nicgpu_device_count",
    "nicgpu_get_device",
    "nicgpu_set_device",
    "nicgpu_malloc",
    "nicgpu_free",
    "nicgpu_host_alloc",
    "nicgpu_host_free",
    "nicgpu_memset_async",
    "nicgpu_memcpy_async",
    "nicgpu_stream_synchronize",
    "nicgpu_stream_create",
    "nicgpu_stream_create_priority",
    "nicgpu_stream_destroy",
    "nicgpu_event_create",
    "nicgpu_event_destroy",
    "nicgpu_event_record",
    "nicgpu_stream_wait_event",
    "nicgpu_rss_create",
    "nicgpu_rss_destroy",
    "nicgpu_rss_set_key",
    "nicgpu_rss_set_key_device",
    "nicgpu_rss_set_table",
    "nicgpu_rss_set_table_device",
    "nicgpu_rss_info",
    "nicgpu_rx_offload",
    "nicgpu_rx_offload_ex",
    "nicgpu_checksum_batch",
    "nicgpu_checksum_batch_split",
    "nicgpu_tso_checksum",
    "nicgpu_segment_gather",
    "nicgpu_segment_gather_from",
    "nicgpu_qp_create",
    "nicgpu_qp_destroy",
    "nicgpu_qp_reserve",
    "nicgpu_qp_bind",
    "nicgpu_qp_plan",
    "nicgpu_qp_plan_on",
    "nicgpu_qp_plan_async",
    "nicgpu_qp_piece_count",
    "nicgpu_qp_check",
    "nicgpu_qp_resolve",
    "nicgpu_qp_resolve_start",
    "nicgpu_qp_resolve_finish",
    "nicgpu_qp_rss_list",
    "nicgpu_rx_offload_count",
    "nicgpu_qp_rss_scatter",
    "nicgpu_qp_group",
    "nicgpu_qp_deliver",
    "nicgpu_qp_deliver_range",
    "nicgpu_icrc_batch",
    "nicgpu_tso_segment",
    "nicgpu_cq_create",
    "nicgpu_cq_destroy",
    "nicgpu_cq_post",
    "nicgpu_cq_state",
    "nicgpu_cq_poll",
    "nicgpu_qp_check_flags",
    "nicgpu_qp_set_segments",
    "nicgpu_qp_segment_results",
    "nicgpu_qp_segment_lists",
    "nicgpu_qp_segment_hits",
    "nicgpu_memcpy_batch",
    "nicgpu_qp_walks",
    "nicgpu_qp_check_async",
    "nicgpu_qp_check_wait",
    "nicgpu_qp_check_bounds",
    "nicgpu_qp_resum",
    "nicgpu_qp_set_deferred_verify",
    "nicgpu_qp_set_delivery_reserve",
    "nicgpu_qp_deferred",
    "nicgpu_qp_verify_fixups_async",
    "nicgpu_event_synchronize",
    "nicgpu_host_register",
    "nicgpu_host_unregister",
    "nicgpu_image_stage",
    "nicgpu_image_writeback",
)

_lib = None


class NicGpuError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libnicgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NicGpuError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in signatures().items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nicgpu_abi_version() != ABI_VERSION:
        raise NicGpuError(f"{path}: ABI version {lib.nicgpu_abi_version()}, this package needs {ABI_VERSION}")
    _lib = lib
    return lib


def signatures() -> dict:
    """ctypes (restype, argtypes) of the C-ABI entry points this package calls,
    one per prototype of include/nicgpu.h (tests/test_abi.py checks the
    argument counts against the header)."""
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    return {
        "nicgpu_abi_version": (i32, []),
        "nicgpu_strerror": (ctypes.c_char_p, [i32]),
        "nicgpu_device_count": (i32, []),
        "nicgpu_rss_create": (i32, [ctypes.POINTER(vp), i32]),
        "nicgpu_rss_destroy": (i32, [vp]),
        "nicgpu_rss_set_key": (i32, [vp, vp, sz, vp]),
        "nicgpu_rss_set_key_device": (i32, [vp, vp, sz, vp]),
        "nicgpu_rss_set_table": (i32, [vp, vp, sz, vp]),
        "nicgpu_rss_set_table_device": (i32, [vp, vp, sz, vp]),
        "nicgpu_rss_info": (i32, [vp, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
        "nicgpu_rx_offload": (i32, [vp, vp, vp, sz, i32, u32, u32, vp, vp, vp, vp, vp]),
        "nicgpu_rx_offload_count": (i32, [vp, vp, vp, sz, vp, i32, u32, u32, vp, vp, vp, vp, vp]),
        "nicgpu_rx_offload_ex": (i32, [vp, vp, vp, sz, i32, u32, u32, vp, vp, vp, vp, vp, vp]),
        "nicgpu_segment_gather": (i32, [vp, ctypes.c_uint64, vp, sz, vp]),
        "nicgpu_segment_gather_from": (i32, [vp, vp, ctypes.c_uint64, vp, sz, vp]),
        "nicgpu_qp_create": (i32, [vp, i32]),
        "nicgpu_qp_destroy": (i32, [vp]),
        "nicgpu_qp_reserve": (i32, [vp, sz, sz, vp]),
        "nicgpu_qp_bind": (i32, [vp, vp, sz, vp, sz, vp]),
        "nicgpu_qp_plan": (i32, [vp, vp, ctypes.c_uint64, sz, ctypes.c_uint64, vp, vp, vp]),
        "nicgpu_qp_plan_on": (i32, [vp, vp, ctypes.c_uint64, sz, ctypes.c_uint64, vp, vp, vp, vp]),
        "nicgpu_qp_plan_async": (i32, [vp, vp, ctypes.c_uint64, sz, ctypes.c_uint64, vp, vp, vp]),
        "nicgpu_qp_piece_count": (i32, [vp, vp]),
        "nicgpu_qp_check": (i32, [vp, ctypes.c_uint64, sz, sz, vp, vp]),
        "nicgpu_qp_resolve": (i32, [vp, ctypes.c_uint64, sz, sz, ctypes.c_uint64, ctypes.c_uint16, vp, vp, vp, vp]),
        "nicgpu_qp_resolve_start": (i32, [vp, ctypes.c_uint64, sz, sz, ctypes.c_uint64, ctypes.c_uint16, vp]),
        "nicgpu_qp_resolve_finish": (i32, [vp, vp, vp, vp, vp]),
        "nicgpu_qp_rss_list": (i32, [vp, sz, vp]),
        "nicgpu_qp_rss_scatter": (i32, [vp, sz, vp]),
        "nicgpu_qp_group": (i32, [vp, sz, sz, vp]),
        "nicgpu_qp_deliver": (i32, [vp, vp, ctypes.c_uint64, sz, vp, i32, u32, u32, vp, vp]),
        "nicgpu_qp_deliver_range": (i32, [vp, vp, ctypes.c_uint64, sz, sz, u32, vp, i32, u32, u32, vp, vp]),
        "nicgpu_icrc_batch": (i32, [vp, vp, sz, i32, vp, vp, vp]),
        "nicgpu_tso_segment": (i32, [vp, vp, vp, vp, vp, vp, sz, vp, ctypes.c_uint64, u32, vp, vp, vp]),
        "nicgpu_checksum_batch": (i32, [vp, vp, sz, vp, vp]),
        "nicgpu_checksum_batch_split": (i32, [vp, vp, sz, vp, vp, vp]),
        "nicgpu_cq_create": (i32, [ctypes.POINTER(vp), i32, sz, sz]),
        "nicgpu_cq_destroy": (i32, [vp]),
        "nicgpu_cq_post": (i32, [vp, vp, vp, vp, vp, sz, vp]),
        "nicgpu_cq_state": (i32, [vp, vp, vp]),
        "nicgpu_cq_poll": (i32, [vp, ctypes.c_uint32, vp, sz, ctypes.POINTER(sz), vp]),
        "nicgpu_stream_create": (i32, [ctypes.POINTER(vp)]),
        "nicgpu_stream_create_priority": (i32, [ctypes.POINTER(vp), i32]),
        "nicgpu_stream_destroy": (i32, [vp]),
        "nicgpu_event_create": (i32, [ctypes.POINTER(vp)]),
        "nicgpu_event_destroy": (i32, [vp]),
        "nicgpu_event_record": (i32, [vp, vp]),
        "nicgpu_stream_wait_event": (i32, [vp, vp]),
        "nicgpu_tso_checksum": (i32, [vp, vp, vp, vp, vp, sz, vp, vp]),
        "nicgpu_qp_check_flags": (i32, [vp, ctypes.c_uint64, sz, sz, u32, vp, vp]),
        "nicgpu_qp_set_segments": (i32, [vp, vp, sz, sz, vp]),
        "nicgpu_qp_segment_results": (i32, [vp, vp, vp]),
        "nicgpu_qp_segment_lists": (i32, [vp, sz, sz, vp, vp]),
        "nicgpu_qp_segment_hits": (i32, [vp, sz, sz, vp, vp]),
        "nicgpu_memcpy_batch": (i32, [vp, sz, vp]),
        "nicgpu_qp_walks": (i32, [vp, vp]),
        "nicgpu_qp_check_async": (i32, [vp, ctypes.c_uint64, sz, sz, ctypes.c_uint, vp]),
        "nicgpu_qp_check_wait": (i32, [vp, vp]),
        "nicgpu_qp_check_bounds": (i32, [vp, vp]),
        "nicgpu_qp_resum": (i32, [vp, vp, ctypes.c_uint64, vp]),
        "nicgpu_qp_set_deferred_verify": (i32, [vp, i32]),
        "nicgpu_qp_set_delivery_reserve": (i32, [vp, i32]),
        "nicgpu_qp_deferred": (i32, [vp, vp]),
        "nicgpu_qp_verify_fixups_async": (i32, [vp, vp, sz, vp]),
        "nicgpu_event_synchronize": (i32, [vp]),
        "nicgpu_host_register": (i32, [vp, sz, ctypes.POINTER(vp), ctypes.POINTER(i32)]),
        "nicgpu_host_unregister": (i32, [vp]),
        "nicgpu_image_stage": (i32, [vp, vp, ctypes.c_uint64, vp, sz, vp]),
        "nicgpu_image_writeback": (i32, [vp, vp, ctypes.c_uint64, vp, sz, vp]),
    }


def _check(status: int, what: str) -> None:
    if status != OK:
        msg = load_library().nicgpu_strerror(status).decode()
        raise NicGpuError(f"{what} failed: {msg} ({status})")


def _ptr(t):
    """Device (or host) data pointer of a tensor, or None."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _stream_ptr(stream):
    if stream is None:
        import torch

        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def device_count() -> int:
    return load_library().nicgpu_device_count()


def desc_pack(offsets, lengths):
    """numpy: pack byte offsets and lengths into the uint64 descriptor format."""
    import numpy as np

    off = np.asarray(offsets, dtype=np.uint64)
    ln = np.asarray(lengths, dtype=np.uint64)
    return off | (ln << np.uint64(DESC_OFFSET_BITS))


class RssContext:
    """Owner of a ``nicgpu_rss_ctx`` (key LUT + indirection table on one GPU)."""

    def __init__(self, device: int = 0):
        import torch

        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(self.lib.nicgpu_rss_create(ctypes.byref(h), device), "nicgpu_rss_create")
        self.handle = h

    def close(self):
        if self.handle:
            self.lib.nicgpu_rss_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_key(self, key: bytes = b"", stream=None):
        buf = (ctypes.c_uint8 * max(1, len(key))).from_buffer_copy(bytes(key) or b"\0")
        _check(
            self.lib.nicgpu_rss_set_key(self.handle, buf, len(key), _stream_ptr(stream)),
            "nicgpu_rss_set_key",
        )

    def set_key_device(self, key_dev, stream=None):
        _check(
            self.lib.nicgpu_rss_set_key_device(
                self.handle, _ptr(key_dev), key_dev.numel(), _stream_ptr(stream)
            ),
            "nicgpu_rss_set_key_device",
        )

    def set_table(self, table=(), stream=None):
        import numpy as np

        arr = np.ascontiguousarray(np.asarray(table, dtype=np.uint16))
        _check(
            self.lib.nicgpu_rss_set_table(
                self.handle,
                arr.ctypes.data_as(ctypes.c_void_p) if arr.size else None,
                arr.size,
                _stream_ptr(stream),
            ),
            "nicgpu_rss_set_table",
        )

    def set_table_device(self, table_dev, stream=None):
        _check(
            self.lib.nicgpu_rss_set_table_device(
                self.handle, _ptr(table_dev), table_dev.numel(), _stream_ptr(stream)
            ),
            "nicgpu_rss_set_table_device",
        )

    def info(self):
        k, t = ctypes.c_size_t(), ctypes.c_size_t()
        _check(self.lib.nicgpu_rss_info(self.handle, ctypes.byref(k), ctypes.byref(t)), "info")
        return k.value, t.value


def rx_offload(ctx, frames, desc, mode=TUPLE_AUTO, raw_off=0, raw_len=0, csum=None,
               hash_out=None, queue=None, hits=None, stream=None, l34=None):
    """Launch the fused RX checksum + RSS kernel on torch device tensors.

    l34 (uint8[n], optional): NICGPU_L34_* flags of the L3/L4 checksum
    verification done in the same pass (nicgpu_rx_offload_ex)."""
    lib = load_library()
    n = desc.numel()
    if l34 is None:
        _check(
            lib.nicgpu_rx_offload(
                ctx.handle if ctx is not None else None,
                _ptr(frames), _ptr(desc), n, mode, raw_off, raw_len,
                _ptr(csum), _ptr(hash_out), _ptr(queue), _ptr(hits), _stream_ptr(stream),
            ),
            "nicgpu_rx_offload",
        )
        return
    _check(
        lib.nicgpu_rx_offload_ex(
            ctx.handle if ctx is not None else None,
            _ptr(frames), _ptr(desc), n, mode, raw_off, raw_len,
            _ptr(csum), _ptr(hash_out), _ptr(queue), _ptr(hits), _ptr(l34), _stream_ptr(stream),
        ),
        "nicgpu_rx_offload_ex",
    )


SEG_TSO = 0x10000
SEG_VLAN_INSERT = 0x20000
SEG_VLAN_STRIP = 0x40000
SEG_VLAN_PRESENT = 0x80000


def tso_segment_counts(lens, hdr_len, mss, flags):
    """Segments nicgpu_tso_segment writes per frame (queue_pair.cpp:212-278):
    1 unsegmented, ceil((L - H) / mss) segmented, 0 for InvalidMss /
    TooManySegments.  Returns (counts int64[n], seg_base uint32[n], total)."""
    L = np.asarray(lens, np.int64)
    H = np.broadcast_to(np.asarray(hdr_len, np.int64), L.shape)
    M = np.broadcast_to(np.asarray(mss, np.int64), L.shape)
    F = np.broadcast_to(np.asarray(flags, np.int64), L.shape)
    seg = ((F & SEG_TSO) != 0) & (M > 0) & (L > M)
    invalid = seg & ((M > 9000) | (H > L))
    split = seg & ~invalid & (H < L)
    cnt = np.where(split, (L - H + np.maximum(M, 1) - 1) // np.maximum(M, 1), 1)
    cnt = np.where(invalid | (cnt > 64), 0, cnt)
    base = np.zeros(L.shape, np.int64)
    if L.size > 1:
        base[1:] = np.cumsum(cnt[:-1])
    return cnt, base.astype(np.uint32), int(cnt.sum())


def tso_segment(frames, desc, hdr_len, mss, seg_base, flags, out, stride, out_len=None, out_csum=None, stream=None):
    """Materialise TSO/GSO segments with VLAN insert/strip (nicgpu_tso_segment)."""
    lib = load_library()
    _check(lib.nicgpu_tso_segment(_ptr(frames), _ptr(desc), _ptr(hdr_len), _ptr(mss), _ptr(seg_base), _ptr(flags),
                                  desc.numel(), _ptr(out), out.numel() * out.element_size(), stride, _ptr(out_len),
                                  _ptr(out_csum), _stream_ptr(stream)), "nicgpu_tso_segment")


ICRC_CALCULATE = 0
ICRC_VERIFY = 1


def icrc_batch(frames, desc, mode=ICRC_CALCULATE, crc=None, ok=None, stream=None):
    """RoCEv2 ICRC (CRC-32C) of every descriptor's span (nicgpu_icrc_batch)."""
    lib = load_library()
    _check(lib.nicgpu_icrc_batch(_ptr(frames), _ptr(desc), desc.numel(), mode, _ptr(crc), _ptr(ok),
                                 _stream_ptr(stream)), "nicgpu_icrc_batch")


def checksum_batch(frames, desc, csum, stream=None):
    lib = load_library()
    _check(
        lib.nicgpu_checksum_batch(_ptr(frames), _ptr(desc), desc.numel(), _ptr(csum),
                                  _stream_ptr(stream)),
        "nicgpu_checksum_batch",
    )


def tso_checksum(frames, desc, hdr_len, mss, seg_base, out, stream=None):
    lib = load_library()
    _check(
        lib.nicgpu_tso_checksum(_ptr(frames), _ptr(desc), _ptr(hdr_len), _ptr(mss),
                                _ptr(seg_base), desc.numel(), _ptr(out), _stream_ptr(stream)),
        "nicgpu_tso_checksum",
    )
