#!/usr/bin/env python3
"""Compare the gfx950 ISA of kernels between two `hipcc --cuda-device-only -S`
outputs (a refactor check: the production kernels must compile to the same
instructions).  Kernels are matched by a demangled-name pattern; labels and
comments are normalised away, and the kernel's VGPR/SGPR/LDS/scratch
metadata is compared too.

  python tools/isa_diff.py before.s after.s deliver_kernel 'rx_offload_kernelILi2ELb1ELi4=rx_offload_kernelILi2ELi4' ...

Exit 0 when every named kernel that exists on both sides is identical."""

import re
import sys


def kernels(path):
    """symbol -> (instructions, metadata) for every .globl function."""
    text = open(path).read().splitlines()
    out, cur, body = {}, None, []
    meta = {}
    for line in text:
        m = re.match(r"^(\S+):\s*(;.*)?$", line)
        if m and not line.startswith(".") and not m.group(1).startswith(".L"):
            if cur is not None:
                out[cur] = body
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if line.strip().startswith(".Lfunc_end"):
            out[cur] = body
            cur, body = None, []
            continue
        s = line.split(";", 1)[0].strip()
        if not s or s.startswith("."):
            continue
        s = re.sub(r"\.LBB\d+_\d+", "L", s)
        body.append(s)
    # metadata from the kernel descriptors: .amdhsa_next_free_vgpr etc.
    cur = None
    for line in text:
        m = re.match(r"\s*\.amdhsa_kernel\s+(\S+)", line)
        if m:
            cur = m.group(1)
            meta[cur] = {}
            continue
        if cur is not None:
            m = re.match(r"\s*\.amdhsa_(next_free_vgpr|next_free_sgpr|group_segment_fixed_size|"
                         r"private_segment_fixed_size|accum_offset)\s+(\S+)", line)
            if m:
                meta[cur][m.group(1)] = m.group(2)
            if ".end_amdhsa_kernel" in line:
                cur = None
    return {k: (v, meta.get(k, {})) for k, v in out.items()}


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    bad = 0
    for arg in sys.argv[3:]:
        # PAT, or LEFT=RIGHT to pair kernels renamed by the refactor (matched
        # in sorted order of their symbols when the names differ)
        pl, _, pr = arg.partition("=")
        pr = pr or pl
        ka = sorted(k for k in a if pl in k)
        kb = sorted(k for k in b if pr in k)
        if not ka or not kb:
            print(f"{arg}: {len(ka)} kernel(s) on the left, {len(kb)} on the right")
            bad += 1
            continue
        pairs = [(k, k) for k in ka if k in b] if pl == pr else list(zip(ka, kb))
        if len(pairs) != len(ka) or len(ka) != len(kb):
            print(f"{arg}: {len(ka)} kernel(s) on the left, {len(kb)} on the right")
            bad += 1
        for ka_, kb_ in pairs:
            ia, ma = a[ka_]
            ib, mb = b[kb_]
            same = ia == ib and ma == mb
            print(f"{'same' if same else 'DIFF'}  {len(ia):6d} vs {len(ib):6d} instr  "
                  f"vgpr {ma.get('next_free_vgpr')} vs {mb.get('next_free_vgpr')}  {ka_[:70]} | {kb_[:70]}")
            bad += 0 if same else 1
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
