"""GPU parity at BASELINE.json's full sizes for C3 and C5 (C2 is in
test_gpu_parity.py::test_full_size_c2_properties).

At these sizes the oracle is too slow for every packet, so each case checks
size-independent properties over the whole batch plus a sampled bit-exact
comparison with the oracle:
  C3  4 M IMIX 64/576/1518 (7:4:1), 16 queues: status == corruption, queue ==
      table[hash % 128], hits == bincount of the table index (the RssStats
      queue_hits of n sequential select_queue calls, rss.cpp:49-61), determinism.
  C5  131072 x 9000 B, H = 54, mss = 1448 (7 segments): ones'-complement
      linearity between two kernels — for every frame, the segment checksums of
      nicgpu_tso_checksum recombine to the whole-frame checksum of
      nicgpu_rx_offload (checksum.cpp:10-34 sums big-endian words; H and mss
      are even, so every chunk keeps the frame's word alignment):
          sum_k ~cs_k - (nseg - 1) * S(H)  ==  ~cs_frame   (mod 0xFFFF)
      where S(H) is the header's word sum.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import smart_nic_amd as sna  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from smart_nic_amd import pktgen  # noqa: E402

MS_KEY = bytes.fromhex(
    "6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa"
)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    torch.cuda.set_device(0)


def _host(t, dtype):
    return t.cpu().numpy().view(dtype)


def _rx(ctx, f, d, n, tn, mode=sna.TUPLE_AUTO):
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    if mode == sna.TUPLE_NONE:
        sna.checksum_batch(f, d, cs)
        torch.cuda.synchronize()
        return _host(cs, np.uint16), None, None, None
    h = torch.empty(n, dtype=torch.int32, device="cuda")
    q = torch.empty(n, dtype=torch.int16, device="cuda")
    hits = torch.zeros(tn, dtype=torch.int64, device="cuda")
    sna.rx_offload(ctx, f, d, mode, 0, 0, cs, h, q, hits)
    torch.cuda.synchronize()
    return _host(cs, np.uint16), _host(h, np.uint32), _host(q, np.uint16), _host(hits, np.uint64)


def test_full_size_c3_imix_properties():
    """C3: 4 M IMIX packets, 16 queues (table 128 entries i % 16), MS key."""
    n = 4 << 20
    rng = np.random.default_rng(33)
    frames, desc, corrupted = pktgen.make_batch(pktgen.imix_lengths(n, rng), seed=33, proto=6, corrupt_frac=0.01)
    table = (np.arange(128) % 16).astype(np.uint16)
    ctx = sna.RssContext(0)
    ctx.set_key(MS_KEY)
    ctx.set_table(table)
    f = torch.from_numpy(np.concatenate([frames, np.zeros(64, np.uint8)])).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    cs, h, q, hits = _rx(ctx, f, d, n, 128)
    np.testing.assert_array_equal(cs != 0, corrupted)
    np.testing.assert_array_equal(q, table[h % 128])
    np.testing.assert_array_equal(hits, np.bincount(h % 128, minlength=128).astype(np.uint64))
    assert int(hits.sum()) == n
    idx = np.sort(np.random.default_rng(1).choice(n, 4096, replace=False))
    cs_o, h_o, q_o, _, _ = po.rx_batch(frames, desc[idx], MS_KEY, table)
    np.testing.assert_array_equal(cs[idx], cs_o)
    np.testing.assert_array_equal(h[idx], h_o)
    np.testing.assert_array_equal(q[idx], q_o)
    cs2, h2, q2, hits2 = _rx(ctx, f, d, n, 128)
    np.testing.assert_array_equal(cs2, cs)
    np.testing.assert_array_equal(h2, h)
    np.testing.assert_array_equal(hits2, hits)
    ctx.close()


def _be_word_sum(rows):
    """Big-endian 16-bit word sums of each row (even row length)."""
    w = rows.reshape(rows.shape[0], -1, 2).astype(np.uint64)
    return (w[:, :, 0] * 256 + w[:, :, 1]).sum(axis=1)


def test_full_size_c5_tso_linearity():
    """C5: 131072 x 9000 B, H = 54, mss = 1448 -> 7 segment checksums per frame."""
    n, L, H, M = 131072, 9000, 54, 1448
    nseg = (L - H + M - 1) // M
    assert nseg == 7
    rng = np.random.default_rng(55)
    frames = rng.integers(0, 256, n * L + 64, dtype=np.uint8)
    offs = np.arange(n, dtype=np.int64) * L
    desc = sna.desc_pack(offs, np.full(n, L))
    f = torch.from_numpy(frames).cuda()
    d = torch.from_numpy(desc.view(np.int64)).cuda()
    base = (np.arange(n, dtype=np.uint32) * nseg).astype(np.uint32)
    out = torch.full((n * nseg,), -1, dtype=torch.int16, device="cuda")
    sna.tso_checksum(f, d, torch.from_numpy(np.full(n, H, np.uint16)).cuda(),
                     torch.from_numpy(np.full(n, M, np.uint16)).cuda(), torch.from_numpy(base).cuda(), out)
    torch.cuda.synchronize()
    seg = _host(out, np.uint16).reshape(n, nseg).astype(np.int64)
    cs_frame, *_ = _rx(None, f, d, n, 0, mode=sna.TUPLE_NONE)
    s_h = _be_word_sum(frames[: n * L].reshape(n, L)[:, :H]).astype(np.int64)
    lhs = ((0xFFFF - seg).sum(axis=1) - (nseg - 1) * s_h) % 0xFFFF
    rhs = (0xFFFF - cs_frame.astype(np.int64)) % 0xFFFF
    np.testing.assert_array_equal(lhs, rhs)
    # sampled bit-exact comparison with the oracle
    for i in np.random.default_rng(2).choice(n, 64, replace=False):
        k, exp = po.tso_segment_checksums(frames[offs[i]: offs[i] + L].tobytes(), H, M)
        assert k == nseg
        assert seg[i].astype(np.uint16).tolist() == list(exp), int(i)


@pytest.mark.gpu
@pytest.mark.parametrize("wl,desc", [("c3", "host"), ("c5", "host"), ("c3", "dev"), ("c5", "dev keep")])
def test_f1_full_size_device_vs_host(tmp_path, wl, desc):
    """Row f1 at the bench sizes (tools/bench_rx_stage.cpp): 1 M IMIX TX
    descriptors (C3) and 131072 x 9000 B TSO frames (C5, every packet ending at
    its first segment's checksum: positions settle by relaxation without a host
    tail).  The device resolve must equal the host resolve in every
    completion, stat, memory byte and RSS dispatch list.  `dev`: the
    descriptors handed over in device memory (DeviceDescriptors); `keep`: the
    results left there (results_on_device) and copied down to compare."""
    import subprocess

    from test_host_cpp import _build

    exe = _build(tmp_path, "rx_stage_gpu_fuzz")
    r = subprocess.run([exe, "full", wl] + [a for a in desc.split() if a != "host"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert f"full {wl}: ok" in r.stdout
    print(r.stdout.strip())
