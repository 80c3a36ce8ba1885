"""Synthetic RX batches for parity tests and bench.py (host side, numpy).

Frames follow the reference PacketGenerator layout (src/packet_generator.cpp:
46-166): Ethernet (dst MAC, src MAC, ethertype 0x0800) | IPv4 (IHL 5, valid
header checksum, :200-232) | TCP (20 B) or UDP (8 B) with a valid pseudo-header
checksum (:240-305) | random payload.  The RX verify of the reference
(queue_pair.cpp:437-438) checks the ones'-complement sum of the WHOLE frame, so
a frame that should pass carries a balancing word in src-MAC bytes 10..11
(covered by no L3/L4 checksum), making compute_checksum(frame) == 0.  A chosen
fraction of frames then gets one flipped payload byte (status ChecksumError).

Batches are packed: frame i at a 16-B aligned offset, lengths arbitrary; the
bytes between frames are random (the kernels must ignore them).
"""

from __future__ import annotations

import numpy as np

IMIX_SIZES = (64, 576, 1518)
IMIX_WEIGHTS = (7, 4, 1)


def imix_lengths(n: int, rng: np.random.Generator) -> np.ndarray:
    """IMIX 64/576/1518 at 7:4:1, shuffled."""
    w = np.asarray(IMIX_WEIGHTS, dtype=np.float64)
    cls = rng.choice(len(IMIX_SIZES), size=n, p=w / w.sum())
    return np.asarray(IMIX_SIZES, dtype=np.int64)[cls]


def _fold(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    while True:
        hi = s >> np.uint64(16)
        if not hi.any():
            return s
        s = (s & np.uint64(0xFFFF)) + hi


def _range_sums(frames: np.ndarray, starts: np.ndarray, lens: np.ndarray, chunk: int = 1 << 16) -> np.ndarray:
    """Big-endian 16-bit word sums of frames[starts[i] : starts[i]+lens[i]] for
    even starts (odd trailing byte = high byte), as uint64."""
    n = starts.size
    out = np.zeros(n, dtype=np.uint64)
    assert np.all(starts % 2 == 0)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        s0 = int(starts[a])
        e0 = int((starts[b - 1] + lens[b - 1] + 1) // 2 * 2)
        e0 = max(e0, s0)
        seg = frames[s0:e0]
        words = seg.view(">u2").astype(np.uint64)
        cs = np.concatenate([np.zeros(1, np.uint64), np.cumsum(words, dtype=np.uint64)])
        st = (starts[a:b] - s0) // 2
        full = lens[a:b] // 2
        out[a:b] = cs[st + full] - cs[st]
        odd = (lens[a:b] % 2) == 1
        if odd.any():
            last = frames[starts[a:b][odd] + lens[a:b][odd] - 1].astype(np.uint64)
            out[a:b][odd] += last << np.uint64(8)
    return out


def _put16(frames, pos, val):
    val = np.asarray(val, dtype=np.uint64)
    frames[pos] = ((val >> np.uint64(8)) & np.uint64(0xFF)).astype(np.uint8)
    frames[pos + 1] = (val & np.uint64(0xFF)).astype(np.uint8)


def make_batch(lengths, seed: int = 42, proto: int = 6, corrupt_frac: float = 0.01, align: int = 16):
    """Build a packed batch.

    Returns (frames uint8[total], desc uint64[n], corrupted bool[n]).
    lengths: int array (each >= 54 for TCP / >= 42 for UDP gets full headers;
    shorter frames are random bytes).
    """
    rng = np.random.default_rng(seed)
    lens = np.asarray(lengths, dtype=np.int64)
    n = lens.size
    slots = (lens + align - 1) // align * align
    offs = np.zeros(n, dtype=np.int64)
    if n > 1:
        offs[1:] = np.cumsum(slots[:-1])
    total = int(offs[-1] + slots[-1]) + 64 if n else 64
    frames = np.frombuffer(rng.bytes(total), dtype=np.uint8).copy()

    l4len = 20 if proto == 6 else 8
    full = lens >= 34 + l4len
    o = offs[full]
    L = lens[full]
    # Ethernet: ethertype IPv4
    _put16(frames, o + 12, 0x0800)
    # IPv4 header (offset 14)
    frames[o + 14] = 0x45
    frames[o + 15] = 0
    _put16(frames, o + 16, L - 14)
    _put16(frames, o + 20, 0x4000)
    frames[o + 22] = 64
    frames[o + 23] = proto
    _put16(frames, o + 24, 0)
    ip_hdr = frames[(o + 14)[:, None] + np.arange(20)[None, :]].astype(np.uint64)
    ip_sum = _fold((ip_hdr[:, 0::2] << np.uint64(8)).sum(1) + ip_hdr[:, 1::2].sum(1))
    _put16(frames, o + 24, (~ip_sum) & np.uint64(0xFFFF))
    # L4 header (offset 34)
    seglen = (L - 34).astype(np.uint64)
    if proto == 6:
        frames[o + 46] = 0x50
        frames[o + 47] = 0x18
        _put16(frames, o + 50, 0)
        _put16(frames, o + 52, 0)
        cso = o + 50
    else:
        _put16(frames, o + 38, seglen)
        _put16(frames, o + 40, 0)
        cso = o + 40
    src = frames[(o + 26)[:, None] + np.arange(8)[None, :]].astype(np.uint64)
    pseudo = (src[:, 0::2] << np.uint64(8)).sum(1) + src[:, 1::2].sum(1) + np.uint64(proto) + seglen
    l4 = _range_sums(frames, o + 34, L - 34)
    l4c = (~_fold(pseudo + l4)) & np.uint64(0xFFFF)
    if proto == 17:
        l4c = np.where(l4c == 0, np.uint64(0xFFFF), l4c)  # packet_generator.cpp:304
    _put16(frames, cso, l4c)

    # Whole-frame balancing word in src-MAC bytes 10..11.
    _put16(frames, offs + 10, 0)
    rest = _fold(_range_sums(frames, offs, lens))
    w = np.uint64(0xFFFF) - rest
    w = np.where((w == 0) | (rest == 0), np.uint64(0xFFFF), w)
    ok_len = lens >= 12
    _put16(frames, offs[ok_len] + 10, w[ok_len])

    # Corrupt a fraction: flip one byte past the headers.
    corrupted = np.zeros(n, dtype=bool)
    if corrupt_frac > 0 and n:
        k = int(round(corrupt_frac * n))
        cand = np.nonzero(lens >= 60)[0]
        if k and cand.size:
            pick = rng.choice(cand, size=min(k, cand.size), replace=False)
            pos = offs[pick] + 54 + (rng.integers(0, 1 << 30, size=pick.size) % (lens[pick] - 54))
            frames[pos] ^= np.uint8(0x5A)
            corrupted[pick] = True

    desc = offs.astype(np.uint64) | (lens.astype(np.uint64) << np.uint64(40))
    return frames, desc, corrupted
