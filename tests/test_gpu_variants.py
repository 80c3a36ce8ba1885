"""Every RX kernel variant of the tuning build (libnicgpu_tune.so: the
production kernel plus the candidates tools/tune_rx.py times) against the
golden fixtures and the oracle, so that a variant can be promoted to
production only once it is known to be bit-exact.  GPU only."""

import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

torch = pytest.importorskip("torch")

import smart_nic_amd as sna  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from smart_nic_amd import golden, pktgen  # noqa: E402

pytestmark = pytest.mark.gpu

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


@pytest.fixture(scope="module")
def tune():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path = os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so")
    if not os.path.exists(path):
        pytest.fail("libnicgpu_tune.so missing: run __graft_entry__.build()")
    tl = ctypes.CDLL(path)
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    tl.nicgpu_tune_num_variants.restype = i32
    tl.nicgpu_tune_variant_name.restype = ctypes.c_char_p
    tl.nicgpu_tune_variant_name.argtypes = [i32]
    tl.nicgpu_tune_rx_offload.restype = i32
    tl.nicgpu_tune_rx_offload.argtypes = [i32, vp, vp, vp, sz, i32, u32, u32, vp, vp, vp, vp, vp]
    tl.nicgpu_rss_create.argtypes = [ctypes.POINTER(vp), i32]
    tl.nicgpu_rss_set_key.argtypes = [vp, vp, sz, vp]
    tl.nicgpu_rss_set_table.argtypes = [vp, vp, sz, vp]
    tl.nicgpu_rss_destroy.argtypes = [vp]
    torch.cuda.set_device(0)
    return tl


def run_variant(tl, v, frames, desc, key, table, mode=sna.TUPLE_AUTO, raw_off=0, raw_len=0):
    n = desc.size
    h = ctypes.c_void_p()
    assert tl.nicgpu_rss_create(ctypes.byref(h), 0) == 0
    kb = (ctypes.c_uint8 * max(len(key), 1)).from_buffer_copy(key or b"\0")
    assert tl.nicgpu_rss_set_key(h, kb, len(key), None) == 0
    tab = np.ascontiguousarray(table, np.uint16)
    assert tl.nicgpu_rss_set_table(h, tab.ctypes.data, tab.size, None) == 0
    f = torch.from_numpy(np.concatenate([frames, np.zeros(64, np.uint8)])).cuda()
    d = torch.from_numpy(np.ascontiguousarray(desc).view(np.int64)).cuda()
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    hs = torch.empty(n, dtype=torch.int32, device="cuda")
    qs = torch.empty(n, dtype=torch.int16, device="cuda")
    tn = max(tab.size, 128) if tab.size else 128
    hits = torch.zeros(tn, dtype=torch.int64, device="cuda")
    rss = mode != sna.TUPLE_NONE
    st = tl.nicgpu_tune_rx_offload(v, h if rss else None, f.data_ptr(), d.data_ptr(), n, mode, raw_off, raw_len,
                                   cs.data_ptr(), hs.data_ptr() if rss else None, qs.data_ptr() if rss else None,
                                   hits.data_ptr() if rss else None, None)
    torch.cuda.synchronize()
    tl.nicgpu_rss_destroy(h)
    assert st == 0, f"variant {v}: status {st}"
    return (cs.cpu().numpy().view(np.uint16), hs.cpu().numpy().view(np.uint32), qs.cpu().numpy().view(np.uint16),
            hits.cpu().numpy().view(np.uint64))


def _layouts():
    """(name, frames, desc): golden mix, packed unaligned, scattered, IMIX."""
    out = []
    frames, desc, _, _ = golden.rx_mix()
    out.append(("rx_mix", frames, desc))
    rng = np.random.default_rng(77)
    n = 3000
    lens = rng.integers(0, 3000, n)
    offs = np.zeros(n, np.int64)
    nxt = 0
    for i in range(n):
        offs[i] = nxt * 16 + int(rng.integers(0, 16))
        if lens[i]:
            nxt = (offs[i] + lens[i] - 1) // 16 + 1
    fr = rng.integers(0, 256, int(nxt * 16 + 64), dtype=np.uint8)
    out.append(("packed_unaligned", fr, sna.desc_pack(offs, lens)))
    perm = rng.permutation(n)
    out.append(("scattered", fr, sna.desc_pack(offs[perm], lens[perm])))
    f2, d2, _ = pktgen.make_batch(pktgen.imix_lengths(20000, rng), seed=5, proto=17)
    out.append(("imix", f2, d2))
    return out


def test_every_variant_bit_exact(tune):
    nv = tune.nicgpu_tune_num_variants()
    names = [tune.nicgpu_tune_variant_name(i).decode() for i in range(nv)]
    # "*_xc": timing-only experiments without the general (non-contiguous) path
    live = [v for v in range(nv) if not names[v].endswith("_xc")]
    table = (np.arange(128) % 16).astype(np.uint16)
    for name, frames, desc in _layouts():
        cs_o, h_o, q_o, _, hits_o = po.rx_batch(frames, desc, MS_KEY, table)
        for v in live:
            cs, h, q, hits = run_variant(tune, v, frames, desc, MS_KEY, table)
            np.testing.assert_array_equal(cs, cs_o, err_msg=f"{names[v]} {name} csum")
            np.testing.assert_array_equal(h, h_o, err_msg=f"{names[v]} {name} hash")
            np.testing.assert_array_equal(q, q_o, err_msg=f"{names[v]} {name} queue")
            np.testing.assert_array_equal(hits, hits_o, err_msg=f"{names[v]} {name} hits")
        # checksum-only launches take the no-staging layout
        for v in live:
            cs, *_ = run_variant(tune, v, frames, desc, MS_KEY, table, mode=sna.TUPLE_NONE)
            np.testing.assert_array_equal(cs, cs_o, err_msg=f"{names[v]} {name} csum-only")
