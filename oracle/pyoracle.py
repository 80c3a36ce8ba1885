"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker — never by the product path (smart_nic_amd/ does not import it).

  liboracle.so   the C restatement of the reference (oracle.c)
  _ref/libref.so the compiled reference itself (only where it was built; it is
                 built in the container that has /root/reference and travels
                 to the GPU box as a prebuilt file)
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

TUPLE_NONE, TUPLE_AUTO, TUPLE_RAW = 0, 1, 2

_o = None
_r = None


def _vp(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def lib():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"{ORACLE_SO} missing: run `make -C oracle`")
        L = ctypes.CDLL(ORACLE_SO)
        vp, sz, u16, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_int
        L.oracle_compute_checksum.restype = u16
        L.oracle_compute_checksum.argtypes = [vp, sz]
        L.oracle_toeplitz.restype = u32
        L.oracle_toeplitz.argtypes = [vp, sz, vp, sz]
        L.oracle_select_queue.restype = u16
        L.oracle_select_queue.argtypes = [vp, sz, vp, sz, vp, sz, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.oracle_default_key.restype = None
        L.oracle_default_key.argtypes = [vp]
        L.oracle_extract_tuple.restype = sz
        L.oracle_extract_tuple.argtypes = [vp, sz, i32, sz, sz, vp]
        L.oracle_rx_batch.restype = None
        L.oracle_rx_batch.argtypes = [vp, vp, sz, i32, sz, sz, vp, sz, vp, sz, vp, vp, vp, vp, vp]
        L.oracle_tso_segment_checksums.restype = i32
        L.oracle_tso_segment_checksums.argtypes = [vp, sz, u16, u16, i32, vp, sz]
        L.oracle_l34_verify.restype = ctypes.c_uint8
        L.oracle_l34_verify.argtypes = [vp, sz]
        L.oracle_tso_segment.restype = i32
        L.oracle_tso_segment.argtypes = [vp, sz, u16, u16, u32, vp, sz, sz, vp, vp]
        L.oracle_icrc_calculate.restype = u32
        L.oracle_icrc_calculate.argtypes = [vp, sz]
        L.oracle_tso_checksum_batch.restype = sz
        L.oracle_tso_checksum_batch.argtypes = [vp, vp, sz, vp, vp, vp]
        L.oracle_l34_batch.restype = None
        L.oracle_l34_batch.argtypes = [vp, vp, sz, vp]
        L.oracle_icrc_batch.restype = None
        L.oracle_icrc_batch.argtypes = [vp, vp, sz, vp]
        L.oracle_icrc_verify.restype = i32
        L.oracle_icrc_verify.argtypes = [vp, sz]
        _o = L
    return _o


def ref_lib():
    """The compiled reference (None when _ref/libref.so was not built)."""
    global _r
    if _r is None and os.path.exists(REF_SO):
        R = ctypes.CDLL(REF_SO)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        R.ref_compute_checksum.restype = ctypes.c_uint16
        R.ref_compute_checksum.argtypes = [vp, sz]
        R.ref_toeplitz.restype = ctypes.c_uint32
        R.ref_toeplitz.argtypes = [vp, sz, vp, sz]
        R.ref_rx_batch.restype = ctypes.c_uint64
        R.ref_rx_batch.argtypes = [vp, vp, sz, ctypes.c_int, vp, sz, vp, sz, vp, vp, ctypes.c_int]
        _r = R
    return _r


def _buf(b: bytes):
    return np.frombuffer(bytes(b) or b"\0", dtype=np.uint8)


def compute_checksum(data: bytes) -> int:
    a = _buf(data)
    return lib().oracle_compute_checksum(_vp(a), len(data))


def toeplitz(key: bytes, data: bytes) -> int:
    k, d = _buf(key), _buf(data)
    return lib().oracle_toeplitz(_vp(k), len(key), _vp(d), len(data))


def default_key() -> bytes:
    out = np.zeros(20, dtype=np.uint8)
    lib().oracle_default_key(_vp(out))
    return out.tobytes()


def select_queue(key: bytes, table, data: bytes):
    k, d = _buf(key), _buf(data)
    t = np.ascontiguousarray(np.asarray(table, dtype=np.uint16))
    h, i = ctypes.c_uint32(), ctypes.c_uint32()
    q = lib().oracle_select_queue(_vp(k), len(key), _vp(t), t.size, _vp(d), len(data),
                                  ctypes.byref(h), ctypes.byref(i))
    return q, h.value, i.value


def extract_tuple(frame: bytes, mode=TUPLE_AUTO, raw_off=0, raw_len=0) -> bytes:
    f = _buf(frame)
    out = np.zeros(64, dtype=np.uint8)
    n = lib().oracle_extract_tuple(_vp(f), len(frame), mode, raw_off, raw_len, _vp(out))
    return out[:n].tobytes()


def rx_batch(frames: np.ndarray, desc: np.ndarray, key: bytes, table, mode=TUPLE_AUTO,
             raw_off=0, raw_len=0):
    """Whole-batch restatement: returns (csum, hash, queue, tidx, hits)."""
    n = desc.size
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    t = np.ascontiguousarray(np.asarray(table, dtype=np.uint16))
    k = _buf(key)
    csum = np.zeros(n, np.uint16)
    hsh = np.zeros(n, np.uint32)
    q = np.zeros(n, np.uint16)
    tidx = np.zeros(n, np.uint32)
    hits = np.zeros(max(1, t.size), np.uint64)
    lib().oracle_rx_batch(_vp(frames), _vp(desc), n, mode, raw_off, raw_len, _vp(k), len(key),
                          _vp(t), t.size, _vp(csum), _vp(hsh), _vp(q), _vp(tidx), _vp(hits))
    return csum, hsh, q, tidx, hits[: t.size]


def tso_segment_checksums(pkt: bytes, hdr_len: int, mss: int, enabled=True):
    p = _buf(pkt)
    out = np.zeros(128, np.uint16)
    r = lib().oracle_tso_segment_checksums(_vp(p), len(pkt), hdr_len, mss, int(enabled), _vp(out), 128)
    return r, out[: max(r, 0)].copy()


def l34_batch(frames: np.ndarray, desc: np.ndarray) -> np.ndarray:
    """oracle_l34_verify for every descriptor."""
    L = lib()
    frames = np.ascontiguousarray(frames, np.uint8)
    base = frames.ctypes.data
    out = np.empty(desc.size, np.uint8)
    for i, d in enumerate(desc.tolist()):
        off, ln = d & ((1 << 40) - 1), d >> 40
        out[i] = L.oracle_l34_verify(ctypes.c_void_p(base + off), ln)
    return out


def icrc_batch(frames: np.ndarray, desc: np.ndarray, verify=False):
    """oracle_icrc_calculate (or _verify) for every descriptor.
    Returns (crc uint32[n], ok uint8[n] or None); in verify mode crc covers all
    but the last 4 bytes (0 below 4 bytes)."""
    L = lib()
    frames = np.ascontiguousarray(frames, np.uint8)
    base = frames.ctypes.data
    crc = np.zeros(desc.size, np.uint32)
    ok = np.zeros(desc.size, np.uint8) if verify else None
    for i, d in enumerate(desc.tolist()):
        off, ln = d & ((1 << 40) - 1), d >> 40
        if verify:
            ok[i] = L.oracle_icrc_verify(ctypes.c_void_p(base + off), ln)
            crc[i] = L.oracle_icrc_calculate(ctypes.c_void_p(base + off), ln - 4) if ln >= 4 else 0
        else:
            crc[i] = L.oracle_icrc_calculate(ctypes.c_void_p(base + off), ln)
    return crc, ok


def tso_segment(pkt: bytes, hdr_len: int, mss: int, flags: int, stride: int = 9224):
    """oracle_tso_segment: (status_or_count, [segment bytes], [csum])."""
    L = lib()
    buf = np.frombuffer(bytes(pkt) + bytes(16), np.uint8)
    out = np.zeros(64 * stride, np.uint8)
    lens = np.zeros(64, np.uint32)
    cs = np.zeros(64, np.uint16)
    k = L.oracle_tso_segment(_vp(buf), len(pkt), hdr_len, mss, flags, _vp(out), stride, 64, _vp(lens), _vp(cs))
    if k <= 0:
        return k, [], []
    return k, [out[i * stride: i * stride + int(lens[i])].tobytes() for i in range(k)], [int(c) for c in cs[:k]]


class CompletionRing:
    """nic::CompletionQueue restated (src/completion_queue.cpp:10-53): a ring of
    `ring_size` entries; post_completion refuses when full (:30-33), stores at
    the producer index, advances it modulo the ring, counts, and rings the
    doorbell with (queue_id, producer index after the post) (:34-41);
    poll_completion returns the entry at the consumer index or None (:45-53)."""

    def __init__(self, ring_size: int, queue_id: int, doorbell=None):
        self.ring = ring_size
        self.queue_id = queue_id
        self.entries = [None] * ring_size
        self.prod = self.cons = self.count = 0
        self.doorbell = doorbell

    def post_completion(self, entry) -> bool:
        if self.count == self.ring:
            return False
        self.entries[self.prod] = entry
        self.prod = (self.prod + 1) % self.ring
        self.count += 1
        if self.doorbell is not None:
            self.doorbell(self.queue_id, self.prod)
        return True

    def poll_completion(self):
        if self.count == 0:
            return None
        e = self.entries[self.cons]
        self.cons = (self.cons + 1) % self.ring
        self.count -= 1
        return e
