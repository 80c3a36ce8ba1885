#!/usr/bin/env python3
"""Identity of the kernel sources a profile measured.

A committed rocprofv3 summary names the sources it was taken on, so that
bench.py can tell whether its counters still describe this tree:
  rx   the RX kernel's sources (csrc/rx.hip + csrc/common.h): the headline
       roofline traffic (profiles/*_pmc_c2.json)
  all  every GPU source of libnicgpu.so (csrc/*.hip and csrc/*.h, not the
       tuning-only tune.hip): the per-row profile (profiles/*_rows_prof.json)

  python tools/kernel_sha.py rx|all     prints "<sha256> <set>" (sha256sum style)
"""

import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "smart_nic_amd", "csrc")
SETS = {
    "rx": ["common.h", "rx.hip"],
}


def source_files(which):
    if which in SETS:
        return SETS[which]
    if which == "all":
        return sorted(f for f in os.listdir(CSRC) if (f.endswith(".hip") or f.endswith(".h")) and f != "tune.hip")
    raise ValueError(f"unknown source set {which!r}")


def kernel_source_sha(which):
    """sha256 (hex) over the named files' names and bytes, in order; None if one is missing."""
    h = hashlib.sha256()
    try:
        for name in source_files(which):
            with open(os.path.join(CSRC, name), "rb") as f:
                data = f.read()
            h.update(name.encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    except OSError:
        return None
    return h.hexdigest()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    print(f"{kernel_source_sha(which)} {which}")
