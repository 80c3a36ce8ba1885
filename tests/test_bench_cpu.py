"""The CPU legs bench.py reports beside the GPU rows (cpu_baseline.other_rows):
the reference QueuePair driver (oracle/_ref/ref_qp_bench, rows f1 and f2) on a
tiny batch, and the batch form of the L3/L4 restatement (row f3) against its
per-frame form.  Test infrastructure only; no GPU."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

QP_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_qp_bench")


@pytest.mark.skipif(not os.path.exists(QP_BENCH), reason="oracle/_ref/ref_qp_bench not built (needs /root/reference)")
@pytest.mark.parametrize("mode,row,success_per_tx", [("c3", "f1_c3", 1), ("c5seg", "tso_seg_c5", 7), ("c5", "f1_c5", 0)])
def test_ref_qp_bench_rows(mode, row, success_per_tx):
    r = subprocess.run([QP_BENCH, "256", "1", mode], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["row"] == row and d["kind"] == "reference" and d["cores"] == 1 and d["value"] > 0
    # C3 frames are balanced so every RX verify passes; C5 with RX verify off
    # delivers all 7 segments of every frame; with it on, random segments fail
    assert d["rx_success"] == 256 * success_per_tx


def test_l34_batch_matches_per_frame():
    import ctypes

    from oracle import pyoracle as po
    from smart_nic_amd import pktgen

    L = po.lib()
    lens = np.random.default_rng(5).integers(20, 1600, 400)
    frames, desc, _ = pktgen.make_batch(lens, seed=5, proto=6, corrupt_frac=0.1)
    out = np.zeros(desc.size, np.uint8)
    vp = ctypes.c_void_p
    L.oracle_l34_batch(vp(frames.ctypes.data), vp(desc.ctypes.data), desc.size, vp(out.ctypes.data))
    for i, d in enumerate(desc.tolist()):
        off, n = d & ((1 << 40) - 1), d >> 40
        assert out[i] == L.oracle_l34_verify(vp(frames.ctypes.data + off), n)
