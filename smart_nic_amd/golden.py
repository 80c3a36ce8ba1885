"""Readers for the committed golden fixtures in tests/golden/ (plain data).

The fixtures were produced by oracle/gen_golden.cpp from the compiled
reference (src/checksum.cpp, src/rss.cpp, src/queue_pair.cpp).  This module
only parses them; it never runs anything from the reference.
"""

from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def path(name: str) -> str:
    return os.path.join(GOLDEN_DIR, name)


def load_json(name: str):
    with open(path(name)) as f:
        return json.load(f)


def load_bin(name: str, dtype) -> np.ndarray:
    return np.fromfile(path(name), dtype=dtype)


def hexbytes(s: str) -> bytes:
    return bytes.fromhex(s)


def rx_mix():
    """The mixed-frame fixture: frames, desc, csum and per-config expectations."""
    frames = load_bin("rx_mix.frames.bin", np.uint8)
    desc = load_bin("rx_mix.desc.bin", np.uint64)
    csum = load_bin("rx_mix.csum.bin", np.uint16)
    meta = load_json("rx_mix.json")
    cfgs = []
    for c in meta["configs"]:
        name = c["name"]
        c = dict(c)
        c["key"] = hexbytes(c["key"])
        c["hash"] = load_bin(f"rx_mix.{name}.hash.bin", np.uint32)
        c["queue"] = load_bin(f"rx_mix.{name}.queue.bin", np.uint16)
        c["tidx"] = load_bin(f"rx_mix.{name}.tidx.bin", np.uint32)
        cfgs.append(c)
    return frames, desc, csum, cfgs


def checksum_sweep():
    return (
        load_bin("checksum_sweep.frames.bin", np.uint8),
        load_bin("checksum_sweep.desc.bin", np.uint64),
        load_bin("checksum_sweep.csum.bin", np.uint16),
    )


def c1():
    return (
        load_bin("c1_udp64.frames.bin", np.uint8),
        load_bin("c1_udp64.desc.bin", np.uint64),
        load_json("c1_udp64.json"),
    )


def tso():
    return load_bin("tso.frames.bin", np.uint8), load_json("tso.json")


def l34():
    """L3/L4 verification fixture: frames, desc, expected flags."""
    return (
        load_bin("l34.frames.bin", np.uint8),
        load_bin("l34.desc.bin", np.uint64),
        load_bin("l34.flags.bin", np.uint8),
    )
