"""GPU parity: the HIP path (through the C-ABI of include/nicgpu.h) against the
reference's golden fixtures and the CPU oracle.  Bit-exact for every output.

Runs on a real MI355X only (marker `gpu`).  Sizes are chosen so the oracle
finishes in seconds; the full-size (1 M x 1518 B) case is checked through
size-independent properties plus a sampled oracle comparison.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import smart_nic_amd as sna  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from smart_nic_amd import golden, pktgen  # noqa: E402

MS_KEY = bytes.fromhex(
    "6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa"
)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert sna.device_count() >= 1, "no gfx950 device visible to libnicgpu.so"
    torch.cuda.set_device(0)
    yield
    torch.cuda.synchronize()


def dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    elif a.dtype == np.uint16:
        a = a.view(np.int16)
    return torch.from_numpy(a).cuda()


def host(t, dtype):
    return t.cpu().numpy().view(dtype)


def gpu_rx(frames, desc, key=b"", table=(), mode=sna.TUPLE_AUTO, raw_off=0, raw_len=0):
    n = desc.size
    ctx = None
    if mode != sna.TUPLE_NONE:
        ctx = sna.RssContext(0)
        ctx.set_key(key)
        ctx.set_table(table)
    f = dev(np.concatenate([frames, np.zeros(64, np.uint8)]))
    d = dev(desc)
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    if mode == sna.TUPLE_NONE:
        sna.checksum_batch(f, d, cs)
        torch.cuda.synchronize()
        return host(cs, np.uint16), None, None, None
    tn = ctx.info()[1]
    h = torch.empty(n, dtype=torch.int32, device="cuda")
    q = torch.empty(n, dtype=torch.int16, device="cuda")
    hits = torch.zeros(tn, dtype=torch.int64, device="cuda")
    sna.rx_offload(ctx, f, d, mode, raw_off, raw_len, cs, h, q, hits)
    torch.cuda.synchronize()
    out = host(cs, np.uint16), host(h, np.uint32), host(q, np.uint16), host(hits, np.uint64)
    # the same batch without checksums takes the header-only kernel
    # (rss_only_kernel): hash, queue and hits must not change
    h2 = torch.empty(n, dtype=torch.int32, device="cuda")
    q2 = torch.empty(n, dtype=torch.int16, device="cuda")
    hits2 = torch.zeros(tn, dtype=torch.int64, device="cuda")
    sna.rx_offload(ctx, f, d, mode, raw_off, raw_len, None, h2, q2, hits2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(h2, np.uint32), out[1], err_msg="header-only RSS: hash")
    np.testing.assert_array_equal(host(q2, np.uint16), out[2], err_msg="header-only RSS: queue")
    np.testing.assert_array_equal(host(hits2, np.uint64), out[3], err_msg="header-only RSS: hits")
    ctx.close()
    return out


def test_checksum_sweep_golden():
    frames, desc, csum = golden.checksum_sweep()
    cs, *_ = gpu_rx(frames, desc, mode=sna.TUPLE_NONE)
    np.testing.assert_array_equal(cs, csum)


def test_checksum_kats_golden():
    kat = golden.load_json("checksum_kat.json")
    bufs = [bytes.fromhex(c["hex"]) for c in kat["cases"]]
    offs, blob = [], bytearray()
    for b in bufs:
        blob += b"\xA5" * ((-len(blob)) % 16 + 3)  # odd offsets, non-zero gap bytes
        offs.append(len(blob))
        blob += b
    frames = np.frombuffer(bytes(blob) + b"\0" * 32, np.uint8)
    desc = sna.desc_pack(offs, [len(b) for b in bufs])
    cs, *_ = gpu_rx(frames, desc, mode=sna.TUPLE_NONE)
    np.testing.assert_array_equal(cs, [c["csum"] for c in kat["cases"]])


def test_rx_mix_golden_all_configs():
    frames, desc, csum, cfgs = golden.rx_mix()
    for c in cfgs:
        cs, h, q, hits = gpu_rx(frames, desc, c["key"], c["table"], c["mode"], c["raw_off"], c["raw_len"])
        np.testing.assert_array_equal(cs, csum, err_msg=c["name"])
        np.testing.assert_array_equal(h, c["hash"], err_msg=c["name"])
        np.testing.assert_array_equal(q, c["queue"], err_msg=c["name"])
        np.testing.assert_array_equal(hits, np.asarray(c["stats_queue_hits"], np.uint64), err_msg=c["name"])


def test_c1_udp64_golden():
    frames, desc, meta = golden.c1()
    cs, h, q, hits = gpu_rx(frames, desc, bytes.fromhex(meta["key"]), meta["table"])
    np.testing.assert_array_equal(cs, meta["csum"])
    np.testing.assert_array_equal(h, meta["hash"])
    np.testing.assert_array_equal(q, meta["queue"])
    np.testing.assert_array_equal(np.where(cs == 0, 0, 2), meta["rx_status"])
    np.testing.assert_array_equal(hits, np.asarray(meta["stats_queue_hits"], np.uint64))


def test_rss_kats_via_raw_mode():
    """rss_kat.json data strings hashed by the kernel (RAW mode over a frame
    that IS the data) — covers short keys, key wrap, tables of any size."""
    kat = golden.load_json("rss_kat.json")
    for c in kat["cases"]:
        datas = [bytes.fromhex(d) for d in c["data"]]
        datas = [d for d in datas if len(d) <= 64]
        offs, blob = [], bytearray()
        for d in datas:
            blob += b"\x00" * ((-len(blob)) % 16)
            offs.append(len(blob))
            blob += d
        frames = np.frombuffer(bytes(blob) + b"\0" * 32, np.uint8)
        desc = sna.desc_pack(offs, [len(d) for d in datas])
        _, h, q, _ = gpu_rx(frames, desc, bytes.fromhex(c["key"]), c["table"], sna.TUPLE_RAW, 0, 64)
        exp = [c["hash"][i] for i, d in enumerate(c["data"]) if len(bytes.fromhex(d)) <= 64]
        np.testing.assert_array_equal(h, exp, err_msg=c["note"])


def test_tso_golden():
    frames, meta = golden.tso()
    cases = [c for c in meta["cases"] if c["tx_status"] == 0]
    desc = sna.desc_pack([c["off"] for c in cases], [c["len"] for c in cases])
    hdr = np.array([c["hdr"] for c in cases], np.uint16)
    mss = np.array([c["mss"] if c["tso"] else 0 for c in cases], np.uint16)
    nseg = np.array([len(c["seg_csum"]) for c in cases], np.uint32)
    base = np.concatenate([[0], np.cumsum(nseg)[:-1]]).astype(np.uint32)
    out = torch.zeros(int(nseg.sum()), dtype=torch.int16, device="cuda")
    f = dev(np.concatenate([frames, np.zeros(64, np.uint8)]))
    sna.tso_checksum(f, dev(desc), dev(hdr), dev(mss), dev(base), out)
    torch.cuda.synchronize()
    got = host(out, np.uint16)
    exp = np.concatenate([np.asarray(c["seg_csum"], np.uint16) for c in cases])
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("seed", [0, 1])
def test_tso_checksum_random_vs_oracle(seed):
    """nicgpu_tso_checksum on random frames: lengths 0..65535 (frames past
    9 KiB take several load groups), any byte offset, header 0..L, mss 0,
    1..15 (several boundaries per chunk), 16..9000; every segment checksum of
    every frame the oracle accepts (oracle_tso_segment_checksums >= 1)."""
    rng = np.random.default_rng(100 + seed)
    n = 1500
    kind = rng.random(n)
    lens = np.where(kind < 0.15, rng.integers(0, 100, n),
                    np.where(kind < 0.8, rng.integers(100, 9217, n), rng.integers(9217, 65536, n)))
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 40))
        offs[i] = pos
        pos += int(lens[i])
    frames = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    mk = rng.random(n)
    mss = np.where(mk < 0.2, 0, np.where(mk < 0.3, rng.integers(1, 16, n),
                                         np.where(mk < 0.8, rng.integers(16, 1501, n), rng.integers(1501, 9001, n))))
    hdr = np.minimum(rng.integers(0, 200, n), lens)
    exp, nseg = [], np.zeros(n, np.int64)
    for i in range(n):
        pkt = frames[offs[i]: offs[i] + lens[i]].tobytes()
        k, cs = po.tso_segment_checksums(pkt, int(hdr[i]), int(mss[i]))
        exp.append(cs if k >= 1 else None)
        L, H, M = int(lens[i]), int(hdr[i]), int(mss[i])
        seg = M > 0 and L > M and H < L
        nseg[i] = (L - H + M - 1) // M if seg else 1
    base = np.concatenate([[0], np.cumsum(nseg)[:-1]]).astype(np.uint32)
    out = torch.full((int(nseg.sum()),), -1, dtype=torch.int16, device="cuda")
    f = dev(frames)
    sna.tso_checksum(f, dev(sna.desc_pack(offs, lens)), dev(hdr.astype(np.uint16)), dev(mss.astype(np.uint16)),
                     dev(base), out)
    torch.cuda.synchronize()
    got = host(out, np.uint16)
    checked = 0
    for i in range(n):
        if exp[i] is None:
            continue
        g = int(base[i])
        assert got[g: g + len(exp[i])].tolist() == exp[i].tolist(), (i, int(lens[i]), int(hdr[i]), int(mss[i]))
        checked += 1
    assert checked > n // 2


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_layouts_vs_oracle(seed):
    """Random lengths 0..9216 (incl. empty), random byte offsets, n not a
    multiple of 64, random keys/tables; every output vs the oracle."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(1, 3000))
    lens = rng.integers(0, 9217, n)
    small = rng.random(n) < 0.5
    lens[small] = rng.integers(0, 130, int(small.sum()))
    lens[rng.random(n) < 0.4] = rng.choice([0, 1, 13, 14, 33, 34, 54, 60, 64, 65, 576, 1518])
    gaps = rng.integers(0, 40, n)
    offs = np.cumsum(np.concatenate([[gaps[0]], lens[:-1] + gaps[1:]]))
    frames = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    # sprinkle real headers so the parser takes every branch
    pf, pd, _ = pktgen.make_batch(rng.choice([64, 90, 576, 1518], 200), seed=seed, proto=int(rng.choice([6, 17])))
    frames = np.concatenate([frames, pf])
    offs = np.concatenate([offs.astype(np.uint64), (pd & np.uint64((1 << 40) - 1)) + np.uint64(len(frames) - len(pf))])
    lens = np.concatenate([lens, (pd >> np.uint64(40)).astype(np.int64)])
    desc = sna.desc_pack(offs, lens)
    key = rng.integers(0, 256, int(rng.integers(1, 80)), dtype=np.uint8).tobytes()
    table = rng.integers(0, 65536, int(rng.integers(1, 1500))).astype(np.uint16)
    cs_o, h_o, q_o, _, hits_o = po.rx_batch(frames, desc, key, table)
    cs, h, q, hits = gpu_rx(frames, desc, key, table)
    np.testing.assert_array_equal(cs, cs_o)
    np.testing.assert_array_equal(h, h_o)
    np.testing.assert_array_equal(q, q_o)
    np.testing.assert_array_equal(hits, hits_o)


def test_max_packet_and_edge_lengths():
    rng = np.random.default_rng(9)
    lens = np.array([0, 1, 2, 15, 16, 17, 31, 32, 33, 1023, 1024, 1025, 9216, 65535, 65534, 0, 3])
    offs = np.cumsum(np.concatenate([[5], lens[:-1] + 7]))
    frames = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    frames[offs[13]: offs[13] + 65535] = 0xFF  # sum a multiple of 0xFFFF
    desc = sna.desc_pack(offs, lens)
    cs_o, *_ = po.rx_batch(frames, desc, b"", [0], mode=po.TUPLE_NONE)
    cs, *_ = gpu_rx(frames, desc, mode=sna.TUPLE_NONE)
    np.testing.assert_array_equal(cs, cs_o)


def test_default_key_and_table():
    frames, desc, csum, cfgs = golden.rx_mix()
    c = [c for c in cfgs if c["name"] == "default_engine"][0]
    cs, h, q, hits = gpu_rx(frames, desc, b"", ())  # empty key/table -> reference defaults
    np.testing.assert_array_equal(h, c["hash"])
    np.testing.assert_array_equal(q, c["queue"])


def test_set_key_device_matches_host():
    frames, desc, _ = golden.c1()
    ctx = sna.RssContext(0)
    ctx.set_key_device(torch.tensor(list(MS_KEY), dtype=torch.uint8, device="cuda"))
    ctx.set_table_device(torch.tensor([0, 1, 2, 3], dtype=torch.int16, device="cuda"))
    n = desc.size
    f, d = dev(np.concatenate([frames, np.zeros(64, np.uint8)])), dev(desc)
    h = torch.empty(n, dtype=torch.int32, device="cuda")
    q = torch.empty(n, dtype=torch.int16, device="cuda")
    sna.rx_offload(ctx, f, d, sna.TUPLE_AUTO, 0, 0, None, h, q, None)
    torch.cuda.synchronize()
    meta = golden.c1()[2]
    np.testing.assert_array_equal(host(h, np.uint32), meta["hash"])
    np.testing.assert_array_equal(host(q, np.uint16), meta["queue"])


@pytest.mark.parametrize("tn", [16, 128, 4000])
def test_rss_only_imix_vs_oracle(tn):
    """Header-only RSS (no checksum requested) over 200 K IMIX frames at random
    byte offsets with VLAN-tagged, IPv6, fragmented and short frames mixed in;
    tables that fit LDS and one that does not (hits through global atomics);
    hash, queue and hits vs the oracle, and the device-count launch
    (nicgpu_rx_offload_count) over a prefix."""
    rng = np.random.default_rng(tn)
    n = 200_000
    lens = pktgen.imix_lengths(n, rng)
    frames, desc, _ = pktgen.make_batch(lens, seed=tn, proto=6, corrupt_frac=0.0)
    # odd byte offsets for one packet in four: move its bytes 1..15 B later
    offs = (desc & np.uint64((1 << 40) - 1)).astype(np.int64)
    ln = (desc >> np.uint64(40)).astype(np.int64)
    shift = np.where(rng.random(n) < 0.25, rng.integers(1, 16, n), 0)
    blob = np.zeros(len(frames) + 16 * n + 64, np.uint8)
    new_offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos += int(shift[i])
        new_offs[i] = pos
        blob[pos: pos + ln[i]] = frames[offs[i]: offs[i] + ln[i]]
        pos += int(ln[i]) + (-(pos + int(ln[i])) % 16)
    # short and odd frames: truncate some, tag some with 802.1Q, make some IPv6 / fragments
    for i in rng.choice(n, 3000, replace=False):
        k = rng.integers(0, 4)
        o = new_offs[i]
        if k == 0:
            ln[i] = int(rng.integers(0, 40))
        elif k == 1 and ln[i] >= 64:
            blob[o + 12: o + 14] = (0x81, 0x00)
        elif k == 2 and ln[i] >= 64:
            blob[o + 12: o + 14] = (0x86, 0xDD)
            blob[o + 14] = 0x60
        elif ln[i] >= 64:
            blob[o + 20] |= 0x20  # more fragments
    desc2 = sna.desc_pack(new_offs, ln)
    key = bytes(MS_KEY)
    table = rng.integers(0, 16, tn).astype(np.uint16)
    _, h_o, q_o, _, hits_o = po.rx_batch(blob, desc2, key, table)
    ctx = sna.RssContext(0)
    ctx.set_key(key)
    ctx.set_table(table)
    f, d = dev(blob), dev(desc2)
    h = torch.empty(n, dtype=torch.int32, device="cuda")
    q = torch.empty(n, dtype=torch.int16, device="cuda")
    hits = torch.zeros(tn, dtype=torch.int64, device="cuda")
    sna.rx_offload(ctx, f, d, sna.TUPLE_AUTO, 0, 0, None, h, q, hits)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(h, np.uint32), h_o)
    np.testing.assert_array_equal(host(q, np.uint16), q_o)
    np.testing.assert_array_equal(host(hits, np.uint64), hits_o)
    # device-count launch over the first m packets: the rest untouched
    m = 123_457
    lib = sna.load_library()
    n_dev = torch.tensor([m], dtype=torch.int64, device="cuda")
    h.fill_(-1)
    q.fill_(-1)
    hits.zero_()
    assert lib.nicgpu_rx_offload_count(ctx.handle, f.data_ptr(), d.data_ptr(), n, n_dev.data_ptr(), sna.TUPLE_AUTO,
                                       0, 0, None, h.data_ptr(), q.data_ptr(), hits.data_ptr(), None) == sna.OK
    torch.cuda.synchronize()
    hh, qq = host(h, np.uint32), host(q, np.uint16)
    np.testing.assert_array_equal(hh[:m], h_o[:m])
    np.testing.assert_array_equal(qq[:m], q_o[:m])
    assert (hh[m:] == 0xFFFFFFFF).all() and (qq[m:] == 0xFFFF).all()
    np.testing.assert_array_equal(host(hits, np.uint64), np.bincount(h_o[:m] % tn, minlength=tn).astype(np.uint64))
    ctx.close()


def test_invalid_arguments():
    lib = sna.load_library()
    assert lib.nicgpu_rx_offload(None, None, None, 0, 9, 0, 0, None, None, None, None, None) == sna.ERR_INVALID
    ctx = sna.RssContext(0)
    # RAW window beyond the staged header
    assert lib.nicgpu_rx_offload(ctx.handle, None, None, 1, sna.TUPLE_RAW, 60, 8, None, None, None, None, None) == sna.ERR_INVALID
    # empty batch is a no-op
    assert lib.nicgpu_rx_offload(ctx.handle, None, None, 0, sna.TUPLE_AUTO, 0, 0, None, None, None, None, None) == sna.OK


def test_full_size_c2_properties():
    """C2 at full size: 1 M x 1518 B TCP, 1 % corrupted, MS key, table 128 i%4."""
    n = 1 << 20
    frames, desc, corrupted = pktgen.make_batch(np.full(n, 1518), seed=42, proto=6, corrupt_frac=0.01)
    table = np.arange(128) % 4
    cs, h, q, hits = gpu_rx(frames, desc, MS_KEY, table)
    # status property: Success iff the frame was not corrupted
    np.testing.assert_array_equal(cs != 0, corrupted)
    np.testing.assert_array_equal(q, table[h % 128])
    assert int(hits.sum()) == n
    # sampled exact comparison with the oracle
    idx = np.random.default_rng(0).choice(n, 2048, replace=False)
    cs_o, h_o, q_o, _, _ = po.rx_batch(frames, desc[idx], MS_KEY, table)
    np.testing.assert_array_equal(cs[idx], cs_o)
    np.testing.assert_array_equal(h[idx], h_o)
    np.testing.assert_array_equal(q[idx], q_o)
    # determinism
    cs2, h2, q2, hits2 = gpu_rx(frames, desc, MS_KEY, table)
    np.testing.assert_array_equal(cs2, cs)
    np.testing.assert_array_equal(h2, h)
    np.testing.assert_array_equal(hits2, hits)


def test_ring_flushes_small_packets_vs_oracle():
    """2.5 M x 64 B: more tiles per wave than the LDS result ring holds, so the
    production kernel flushes the ring mid-stream (sc1 stores) as well as at
    the end.  Every packet: status and queue properties; a 50 k sample across
    the batch (every flush round): exact vs the oracle; determinism."""
    n = 2_500_000
    frames, desc, corrupted = pktgen.make_batch(np.full(n, 64), seed=11, proto=17, corrupt_frac=0.01)
    table = np.arange(128) % 4
    cs, h, q, hits = gpu_rx(frames, desc, MS_KEY, table)
    np.testing.assert_array_equal(cs != 0, corrupted)
    np.testing.assert_array_equal(q, table[h % 128])
    np.testing.assert_array_equal(hits, np.bincount(h % 128, minlength=128).astype(np.uint64))
    idx = np.sort(np.random.default_rng(1).choice(n, 50_000, replace=False))
    cs_o, h_o, q_o, _, _ = po.rx_batch(frames, desc[idx], MS_KEY, table)
    np.testing.assert_array_equal(cs[idx], cs_o)
    np.testing.assert_array_equal(h[idx], h_o)
    np.testing.assert_array_equal(q[idx], q_o)
    cs2, h2, q2, hits2 = gpu_rx(frames, desc, MS_KEY, table)
    np.testing.assert_array_equal(cs2, cs)
    np.testing.assert_array_equal(h2, h)
    np.testing.assert_array_equal(q2, q)
    np.testing.assert_array_equal(hits2, hits)


def test_imix_16q_vs_oracle():
    rng = np.random.default_rng(3)
    n = 200_000
    frames, desc, corrupted = pktgen.make_batch(pktgen.imix_lengths(n, rng), seed=3, proto=17)
    table = np.arange(128) % 16
    cs, h, q, hits = gpu_rx(frames, desc, MS_KEY, table)
    cs_o, h_o, q_o, _, hits_o = po.rx_batch(frames, desc, MS_KEY, table)
    np.testing.assert_array_equal(cs, cs_o)
    np.testing.assert_array_equal(h, h_o)
    np.testing.assert_array_equal(q, q_o)
    np.testing.assert_array_equal(hits, hits_o)
    np.testing.assert_array_equal(cs != 0, corrupted)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_contiguous_unaligned_layouts_vs_oracle(seed):
    """Packed-in-chunk-space batches (the contiguous-tile fast path): each
    packet starts at a random byte inside the 16-B chunk right after the
    previous packet's last chunk; empty and sub-64-B packets included; random
    bytes in the unused head/tail bytes of every chunk."""
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(60, 5000))
    kind = seed % 4
    if kind == 0:
        lens = rng.integers(0, 3000, n)
    elif kind == 1:
        lens = rng.choice([0, 1, 5, 15, 16, 17, 31, 33, 48, 63, 64, 65], n)
    elif kind == 2:
        lens = rng.integers(900, 9217, n)
    else:
        lens = pktgen.imix_lengths(n, rng)
        lens[rng.random(n) < 0.05] = 0
    offs = np.zeros(n, np.int64)
    nxt = 0  # next free chunk index
    for i in range(n):
        lo = int(rng.integers(0, 16)) if kind != 3 else 0
        offs[i] = nxt * 16 + lo
        if lens[i] > 0:
            nxt = (offs[i] + lens[i] - 1) // 16 + 1
    frames = rng.integers(0, 256, int(nxt * 16 + 64), dtype=np.uint8)
    pf, pd, _ = pktgen.make_batch(np.maximum(lens, 0), seed=seed, proto=6, corrupt_frac=0.02)
    # copy real headers into the packets so the parser sees IPv4/TCP frames
    poff = (pd & np.uint64((1 << 40) - 1)).astype(np.int64)
    for i in range(0, n, 3):
        L = int(lens[i])
        frames[offs[i]: offs[i] + L] = pf[poff[i]: poff[i] + L]
    desc = sna.desc_pack(offs, lens)
    key = MS_KEY if seed % 2 == 0 else bytes(range(1, 21))
    table = (np.arange(128) % 16).astype(np.uint16)
    cs_o, h_o, q_o, _, hits_o = po.rx_batch(frames, desc, key, table)
    cs, h, q, hits = gpu_rx(frames, desc, key, table)
    np.testing.assert_array_equal(cs, cs_o)
    np.testing.assert_array_equal(h, h_o)
    np.testing.assert_array_equal(q, q_o)
    np.testing.assert_array_equal(hits, hits_o)
    cs2, *_ = gpu_rx(frames, desc, mode=sna.TUPLE_NONE)
    np.testing.assert_array_equal(cs2, cs_o)


# ------------------------------------------- L3/L4 verification (§8 f3) --
def gpu_l34(frames, desc, key=None, table=(), mode=sna.TUPLE_NONE):
    n = desc.size
    ctx = None
    if mode != sna.TUPLE_NONE:
        ctx = sna.RssContext(0)
        ctx.set_key(key)
        ctx.set_table(table)
    f = dev(np.concatenate([frames, np.zeros(64, np.uint8)]))
    d = dev(desc)
    cs = torch.empty(n, dtype=torch.int16, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    h = q = None
    if mode != sna.TUPLE_NONE:
        h = torch.empty(n, dtype=torch.int32, device="cuda")
        q = torch.empty(n, dtype=torch.int16, device="cuda")
    sna.rx_offload(ctx, f, d, mode, 0, 0, cs, h, q, None, l34=fl)
    torch.cuda.synchronize()
    out = host(cs, np.uint16), host(fl, np.uint8), None if h is None else host(h, np.uint32)
    if ctx is not None:
        ctx.close()
    return out


@pytest.mark.parametrize("mode", [sna.TUPLE_NONE, sna.TUPLE_AUTO])
def test_l34_golden(mode):
    """Flags pinned by the reference's compute_checksum (tests/golden/l34.*):
    options, VLAN/QinQ, fragments, padding, truncation, bad lengths, UDP
    without checksum, frames at every byte offset.  Checksum and RSS outputs
    of the same launch stay exact."""
    frames, desc, flags = golden.l34()
    cs, fl, h = gpu_l34(frames, desc, MS_KEY, np.arange(128) % 4, mode)
    np.testing.assert_array_equal(fl, flags)
    cs_o, h_o, *_ = po.rx_batch(frames, desc, MS_KEY, np.arange(128) % 4)
    np.testing.assert_array_equal(cs, cs_o)
    if h is not None:
        np.testing.assert_array_equal(h, h_o)


@pytest.mark.parametrize("proto", [6, 17])
def test_l34_generated_batches_vs_oracle(proto):
    """IMIX batches with valid L3/L4 checksums and 2 % corrupted frames."""
    rng = np.random.default_rng(40 + proto)
    n = 60_000
    frames, desc, corrupted = pktgen.make_batch(pktgen.imix_lengths(n, rng), seed=proto, proto=proto,
                                                corrupt_frac=0.02)
    cs, fl, _ = gpu_l34(frames, desc)
    np.testing.assert_array_equal(fl, po.l34_batch(frames, desc))
    ok = sna.L34_IPV4 | sna.L34_IPV4_OK | sna.L34_L4 | sna.L34_L4_OK
    assert ((fl & ok) == ok)[~corrupted].all()


# ------------------------------------------------------- RoCEv2 ICRC (§8 f4) --
def gpu_icrc(frames, desc, verify=False):
    n = desc.size
    f = dev(np.concatenate([frames, np.zeros(64, np.uint8)]))
    d = dev(desc)
    crc = torch.empty(n, dtype=torch.int32, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda") if verify else None
    sna.icrc_batch(f, d, sna.ICRC_VERIFY if verify else sna.ICRC_CALCULATE, crc, ok)
    torch.cuda.synchronize()
    return host(crc, np.uint32), None if ok is None else host(ok, np.uint8)


def test_icrc_published_vectors_gpu():
    kat = golden.load_json("icrc_kat.json")
    blob, offs, lens = bytearray(), [], []
    for c in kat["calculate"]:
        b = bytes.fromhex(c["hex"])
        blob += b"\x5A" * (len(blob) % 3 + 1)  # odd offsets
        offs.append(len(blob))
        lens.append(len(b))
        blob += b
    crc, _ = gpu_icrc(np.frombuffer(bytes(blob), np.uint8), sna.desc_pack(offs, lens))
    np.testing.assert_array_equal(crc, [c["crc"] for c in kat["calculate"]])


@pytest.mark.parametrize("seed", [0, 1])
def test_icrc_random_batches_vs_oracle(seed):
    rng = np.random.default_rng(900 + seed)
    n = 30_000
    lens = np.where(rng.random(n) < 0.1, rng.integers(0, 8, n), pktgen.imix_lengths(n, rng))
    lens[:4] = [0, 65535, 9000, 3]
    gaps = rng.integers(0, 24, n)
    offs = np.cumsum(np.concatenate([[0], (lens + gaps)[:-1]])) + gaps[0]
    frames = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    # a valid big-endian ICRC trailer on every other span
    for i in range(0, n, 2):
        L = int(lens[i])
        if L >= 4:
            c, _ = po.icrc_batch(frames[offs[i]:], np.array([(L - 4) << 40], np.uint64))
            frames[offs[i] + L - 4: offs[i] + L] = np.frombuffer(int(c[0]).to_bytes(4, "big"), np.uint8)
    desc = sna.desc_pack(offs, lens)
    crc, _ = gpu_icrc(frames, desc)
    np.testing.assert_array_equal(crc, po.icrc_batch(frames, desc)[0])
    crc_v, ok = gpu_icrc(frames, desc, verify=True)
    crc_o, ok_o = po.icrc_batch(frames, desc, verify=True)
    np.testing.assert_array_equal(ok, ok_o)
    np.testing.assert_array_equal(crc_v, crc_o)
    assert ok.sum() >= (lens[::2] >= 4).sum()


# --------------------------------------- TSO/GSO + VLAN materialisation (§8 f2) --
def gpu_tso_segment(frames, desc, hdr, mss, flags, stride, fill_seed=None):
    """fill_seed: the output starts as seeded random bytes instead of zeros (the
    kernel rewrites slot bytes past a segment's end up to its 128-B line with
    their own values; those bytes must come back unchanged)."""
    lens = (desc >> np.uint64(40)).astype(np.int64)
    cnt, base, total = sna.tso_segment_counts(lens, hdr, mss, flags)
    f = dev(np.concatenate([frames, np.zeros(64, np.uint8)]))
    nbytes = max(total, 1) * stride
    if fill_seed is None:
        out = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    else:
        out = dev(np.random.default_rng(fill_seed).integers(0, 256, nbytes, dtype=np.uint8))
    ol = torch.zeros(max(total, 1), dtype=torch.int32, device="cuda")
    oc = torch.zeros(max(total, 1), dtype=torch.int16, device="cuda")
    sna.tso_segment(f, dev(desc), dev(np.asarray(hdr, np.uint16)), dev(np.asarray(mss, np.uint16)), dev(base),
                    dev(np.asarray(flags, np.uint32)), out, stride, ol, oc)
    torch.cuda.synchronize()
    return cnt, base, out.cpu().numpy(), host(ol, np.uint32), host(oc, np.uint16)


def test_tso_vlan_segments_golden():
    """Every segment the reference QueuePair delivered (bytes via slot hash,
    checksum, total length) for 160 TSO/GSO + VLAN insert/strip cases."""
    meta = golden.load_json("tso_vlan.json")
    frames = golden.load_bin("tso_vlan.frames.bin", np.uint8)
    cases = meta["cases"]
    desc = sna.desc_pack([c["off"] for c in cases], [c["len"] for c in cases])
    flags = [((sna.SEG_TSO if c["tso"] else 0) | (sna.SEG_VLAN_INSERT if c["insert"] else 0)
              | (sna.SEG_VLAN_STRIP if c["strip"] else 0) | (sna.SEG_VLAN_PRESENT if c["present"] else 0) | c["tag"])
             for c in cases]
    stride = 9216 + 8
    cnt, base, out, ol, oc = gpu_tso_segment(frames, desc, [c["hdr"] for c in cases], [c["mss"] for c in cases],
                                             flags, stride)
    import test_oracle_golden as tog

    for i, c in enumerate(cases):
        want = c["segments"] if c["tx_status"] == 0 else 0
        assert cnt[i] == want
        if not want:
            continue
        g = int(base[i])
        assert int(ol[g:g + want].sum()) == c["rx_bytes"]
        assert oc[g:g + want].tolist() == c["seg_csum"]
        for k in range(want):
            slot = out[(g + k) * stride: (g + k + 1) * stride]
            assert "%x" % tog._fnv(slot.tobytes()) == c["slot_fnv"][k], (i, k)


def test_tso_segment_random_vs_oracle():
    """nicgpu_tso_segment on random frames: lengths 0..20000 (past 9216 B the
    kernel copies from global memory instead of its LDS stage), any byte
    offset, header 0..L+8, mss 0..9100 (incl. < 16 and InvalidMss), random
    VLAN insert / strip / present and tags; every segment's bytes, length and
    checksum vs the oracle, and slot bytes past a segment stay untouched."""
    rng = np.random.default_rng(7)
    n = 600
    lens = np.where(rng.random(n) < 0.85, rng.integers(0, 9300, n), rng.integers(9300, 20001, n))
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 24))
        offs[i] = pos
        pos += int(lens[i])
    frames = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    mk = rng.random(n)
    mss = np.where(mk < 0.1, 0, np.where(mk < 0.2, rng.integers(1, 16, n),
                                         np.where(mk < 0.95, rng.integers(16, 9001, n), rng.integers(9001, 9100, n))))
    hdr = np.minimum(rng.integers(0, 120, n), lens + 8)
    fl = (rng.choice([0, sna.SEG_TSO], n, p=[0.2, 0.8])
          | rng.choice([0, sna.SEG_VLAN_INSERT, sna.SEG_VLAN_STRIP | sna.SEG_VLAN_PRESENT,
                        sna.SEG_VLAN_INSERT | sna.SEG_VLAN_STRIP, sna.SEG_VLAN_STRIP], n)
          | rng.integers(0, 65536, n))
    stride = 20008
    cnt, base, out, ol, oc = gpu_tso_segment(frames, sna.desc_pack(offs, lens), hdr, mss, fl, stride, fill_seed=3)
    fill = np.random.default_rng(3).integers(0, 256, out.size, dtype=np.uint8)
    for i in range(n):
        k, segs, cs = po.tso_segment(frames[offs[i]: offs[i] + lens[i]].tobytes(), int(hdr[i]), int(mss[i]),
                                     int(fl[i]), stride)
        assert max(k, 0) == cnt[i], (i, k, int(cnt[i]))
        g = int(base[i])
        for j in range(max(k, 0)):
            assert ol[g + j] == len(segs[j])
            slot = out[(g + j) * stride: (g + j + 1) * stride]
            assert slot[: len(segs[j])].tobytes() == segs[j], (i, j)
            assert np.array_equal(slot[len(segs[j]):], fill[(g + j) * stride + len(segs[j]): (g + j + 1) * stride]), (i, j)
        assert oc[g: g + max(k, 0)].tolist() == cs


def test_tso_segment_contiguous_run_boundaries():
    """The kernel's one-source path (a segment whose VLAN prefix plus header fit
    64 B is made one contiguous run in its LDS stage) at its edges: prefix +
    header of 63 / 64 / 65 / 68 B (the last two take the two-part copy), mss
    just above, at and below the blob (a later segment's run must not reach
    back into the header), frames starting at every offset 0..15 in their 16-B
    chunk (a first segment's prefix lands before the frame), strip / insert /
    both / neither, slot strides 1506 (segment ends on no 16-B boundary), 1536
    and 1531, random slot fill; every segment vs the oracle, tails untouched."""
    rng = np.random.default_rng(64)
    cases = []
    for hb_target in (63, 64, 65, 68):
        for mode in (sna.SEG_VLAN_INSERT, sna.SEG_VLAN_STRIP | sna.SEG_VLAN_PRESENT,
                     sna.SEG_VLAN_INSERT | sna.SEG_VLAN_STRIP, 0):
            pl = 4 if mode == sna.SEG_VLAN_INSERT else 0
            H = hb_target - pl
            for mss in (hb_target + 1, hb_target, hb_target - 1, 200, 1448):
                for fo in (0, 1, 3, 4, 15):
                    L = int(min(9000, H + 3 * mss + int(rng.integers(0, mss))))
                    cases.append((fo, L, H, mss, sna.SEG_TSO | mode | int(rng.integers(0, 65536))))
    n = len(cases)
    offs = np.zeros(n, np.int64)
    pos = 0
    for i, (fo, L, H, mss, fl) in enumerate(cases):
        pos = (pos + 15) // 16 * 16 + fo
        offs[i] = pos
        pos += L
    frames = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    lens = np.array([c[1] for c in cases], np.int64)
    hdr = np.array([c[2] for c in cases], np.int64)
    mss = np.array([c[3] for c in cases], np.int64)
    fl = np.array([c[4] for c in cases], np.int64)
    segs_seen = 0
    for stride, fill_seed in ((1506, 9), (1536, None), (1531, 11)):
        s_mss = np.minimum(mss, stride - 80)  # every segment fits its slot
        cnt, base, out, ol, oc = gpu_tso_segment(frames, sna.desc_pack(offs, lens), hdr, s_mss, fl, stride, fill_seed)
        fill = (np.zeros(out.size, np.uint8) if fill_seed is None
                else np.random.default_rng(fill_seed).integers(0, 256, out.size, dtype=np.uint8))
        for i in range(n):
            k, segs, cs = po.tso_segment(frames[offs[i]: offs[i] + lens[i]].tobytes(), int(hdr[i]), int(s_mss[i]),
                                         int(fl[i]), stride)
            assert max(k, 0) == cnt[i], (stride, i, k, int(cnt[i]))
            g = int(base[i])
            for j in range(max(k, 0)):
                assert ol[g + j] == len(segs[j])
                slot = out[(g + j) * stride: (g + j + 1) * stride]
                assert slot[: len(segs[j])].tobytes() == segs[j], (stride, i, j)
                assert np.array_equal(slot[len(segs[j]):],
                                      fill[(g + j) * stride + len(segs[j]): (g + j + 1) * stride]), (stride, i, j)
            assert oc[g: g + max(k, 0)].tolist() == cs
            segs_seen += max(k, 0)
    assert segs_seen > 3 * n


@pytest.mark.parametrize("stride,fill_seed", [(1600, None), (1531, 5)])
def test_tso_segment_several_frames_per_wave(stride, fill_seed):
    """16384 frames, so each of the kernel's waves (at most 4096) walks about
    four and the next frame's loads overlap this frame's segments: staged frames
    (0..1500 B) mixed with unstaged ones (9300..9800 B, TSO mss 1448), invalid
    mss, too many segments, frames that do not fit their slot, VLAN variants;
    every segment vs the oracle and slot tails untouched (zeros, or random
    bytes with a stride that is not a multiple of 16)."""
    rng = np.random.default_rng(16)
    n = 16384
    big = rng.random(n) < 0.1
    lens = np.where(big, rng.integers(9300, 9801, n), rng.integers(0, 1501, n))
    offs = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 20))
        offs[i] = pos
        pos += int(lens[i])
    frames = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    mk = rng.random(n)
    mss = np.where(big, 1448, np.where(mk < 0.05, rng.integers(1, 16, n),
                                       np.where(mk < 0.1, rng.integers(9001, 9100, n), rng.integers(100, 1449, n))))
    hdr = np.where(big, 54, np.minimum(rng.integers(0, 120, n), lens + 8))
    fl = (np.where(big | (rng.random(n) < 0.8), sna.SEG_TSO, 0)
          | rng.choice([0, sna.SEG_VLAN_INSERT, sna.SEG_VLAN_STRIP | sna.SEG_VLAN_PRESENT,
                        sna.SEG_VLAN_INSERT | sna.SEG_VLAN_STRIP], n)
          | rng.integers(0, 65536, n))
    cnt, base, out, ol, oc = gpu_tso_segment(frames, sna.desc_pack(offs, lens), hdr, mss, fl, stride, fill_seed)
    fill = (np.zeros(out.size, np.uint8) if fill_seed is None
            else np.random.default_rng(fill_seed).integers(0, 256, out.size, dtype=np.uint8))
    segs_seen = 0
    for i in range(n):
        k, segs, cs = po.tso_segment(frames[offs[i]: offs[i] + lens[i]].tobytes(), int(hdr[i]), int(mss[i]),
                                     int(fl[i]), stride)
        assert max(k, 0) == cnt[i], (i, k, int(cnt[i]))
        g = int(base[i])
        for j in range(max(k, 0)):
            assert ol[g + j] == len(segs[j])
            slot = out[(g + j) * stride: (g + j + 1) * stride]
            assert slot[: len(segs[j])].tobytes() == segs[j], (i, j)
            assert np.array_equal(slot[len(segs[j]):], fill[(g + j) * stride + len(segs[j]): (g + j + 1) * stride]), (i, j)
        assert oc[g: g + max(k, 0)].tolist() == cs
        segs_seen += max(k, 0)
    assert segs_seen > n


def test_tso_segment_c5_vs_oracle():
    """C5 shape (9000 B, H = 54, mss = 1448 and 1447, VLAN variants) at 4096
    frames, unaligned frame offsets; every segment vs the oracle."""
    rng = np.random.default_rng(55)
    n = 4096
    lens = np.full(n, 9000)
    offs = np.arange(n) * 9024 + rng.integers(0, 16, n)
    frames = rng.integers(0, 256, int(offs[-1] + 9000 + 64), dtype=np.uint8)
    mss = np.where(rng.random(n) < 0.5, 1448, 1447)
    hdr = np.where(rng.random(n) < 0.9, 54, 55)
    fl = (sna.SEG_TSO | rng.choice([0, sna.SEG_VLAN_INSERT, sna.SEG_VLAN_STRIP | sna.SEG_VLAN_PRESENT,
                                    sna.SEG_VLAN_INSERT | sna.SEG_VLAN_STRIP], n) | rng.integers(0, 65536, n))
    desc = sna.desc_pack(offs, lens)
    stride = 1536
    cnt, base, out, ol, oc = gpu_tso_segment(frames, desc, hdr, mss, fl, stride, fill_seed=9)
    fill = np.random.default_rng(9).integers(0, 256, out.size, dtype=np.uint8)
    for i in range(0, n, 7):
        k, segs, cs = po.tso_segment(frames[offs[i]: offs[i] + 9000].tobytes(), int(hdr[i]), int(mss[i]), int(fl[i]),
                                     stride)
        assert k == cnt[i]
        g = int(base[i])
        for j in range(k):
            assert ol[g + j] == len(segs[j])
            assert out[(g + j) * stride: (g + j) * stride + len(segs[j])].tobytes() == segs[j]
            lo, hi = (g + j) * stride + len(segs[j]), (g + j + 1) * stride
            assert np.array_equal(out[lo:hi], fill[lo:hi])
        assert oc[g:g + k].tolist() == cs
