"""Per-row kernel measurements for SURVEY §8 beyond the headline line of
bench.py: each row's kernel on its BASELINE/SURVEY configuration, inputs
resident in HBM.  Throughput and roofline come from one HIP event pair around
the K back-to-back launches on the launch stream (as bench.py's line);
us_median is the per-launch median from event pairs in a separate pass.

Rows (SURVEY §8 d configs):
  rx_c2        nicgpu_rx_offload, C2 = 1 M x 1518 B TCP, MS key, table i%4
  rx_l34_c2    the same launch plus L3/L4 verification (f3, nicgpu_rx_offload_ex)
  rx_c3        C3 = 4 M IMIX 64/576/1518 (7:4:1), 16 queues (table i%16)
  icrc_c2      nicgpu_icrc_batch (f4) over the C2 frames
  icrc_c3      nicgpu_icrc_batch over the C3 frames
  rss_c2/rss_c3  hash + queue + hits only (no checksum): the header-only kernel
  tso_c5       nicgpu_tso_checksum, C5 = 131072 x 9000 B, H=54, mss=1448 (7 segments)
  tso_seg_c5   nicgpu_tso_segment (f2): the C5 segments materialised with a VLAN insert,
               plus their checksums

Algorithmic bytes per launch (SURVEY §8 d): sum(L) + 16 N for the RX rows (frame
bytes, 8-B descriptor, 8 B of results); ICRC: sum(L) + 8 N + 4 N; TSO:
sum(L) + 8 N (desc) + 8 N (hdr_len, mss, seg_base) + 2 nseg (checksums).
Prints one JSON object per row on stdout.

  python tools/bench_rows.py [--rows rx_c2,icrc_c2] [--steps 20] [--warmup 3]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
PEAK_GBS = 8000.0


def timed(torch, fn, steps, warmup):
    """(region average, per-launch median) in µs: one HIP event pair around
    `steps` back-to-back launches on the current stream, as bench.py times its
    line (inter-launch gaps included), then per-launch event pairs in a
    separate pass (each pair costs a few µs of wall time per launch)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        fn()
    b.record()
    torch.cuda.synchronize()
    region = a.elapsed_time(b) * 1e3 / steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for x, y in ev:
        x.record()
        fn()
        y.record()
    torch.cuda.synchronize()
    ms = np.array([x.elapsed_time(y) for x, y in ev])
    return region, float(np.median(ms)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="rx_c2,rx_l34_c2,rx_c3,rx_u64,icrc_c2,icrc_c3,tso_c5,tso_seg_c5")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    rows = args.rows.split(",")

    import torch

    import smart_nic_amd as sna
    from smart_nic_amd import pktgen

    torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    cache = {}

    def batch(name):
        if name in cache:
            return cache[name]
        t0 = time.time()
        if name == "c2":
            n = 1 << 20
            frames, desc, _ = pktgen.make_batch(np.full(n, 1518), seed=42, proto=6, corrupt_frac=0.01)
        elif name == "c3":
            n = 4 << 20
            lens = pktgen.imix_lengths(n, np.random.default_rng(33))
            frames, desc, _ = pktgen.make_batch(lens, seed=33, proto=17, corrupt_frac=0.01)
        elif name == "u64":
            n = 4 << 20
            frames, desc, _ = pktgen.make_batch(np.full(n, 64), seed=64, proto=17, corrupt_frac=0.01)
        else:  # c5
            n = 131072
            frames, desc, _ = pktgen.make_batch(np.full(n, 9000), seed=55, proto=6, corrupt_frac=0.0)
        lens = (desc >> np.uint64(40)).astype(np.int64)
        f = torch.from_numpy(frames).to(dev)
        d = torch.from_numpy(desc.view(np.int64)).to(dev)
        cache[name] = (n, int(lens.sum()), f, d)
        print(f"# batch {name}: {n} frames, {lens.sum() / 1e9:.2f} GB in {time.time() - t0:.1f}s", file=sys.stderr)
        return cache[name]

    def rss_ctx(nq):
        ctx = sna.RssContext(dev)
        ctx.set_key(MS_KEY)
        ctx.set_table((np.arange(128) % nq).astype(np.uint16))
        return ctx

    def report(row, workload, n, frame_bytes, alg_bytes, region_us, med_us, extra=None):
        # throughput and roofline from the region average, as bench.py's line
        rec = {"row": row, "workload": workload, "packets": n, "frame_bytes": frame_bytes,
               "alg_bytes_per_launch": alg_bytes, "us_region_avg": round(region_us, 2),
               "us_median": round(med_us, 2),
               "mpkt_s": round(n / region_us, 2), "frame_GBps": round(frame_bytes / region_us / 1e3, 1),
               "alg_GBps": round(alg_bytes / region_us / 1e3, 1),
               "roofline_frac": round(alg_bytes / region_us / 1e3 / PEAK_GBS, 4)}
        if extra:
            rec.update(extra)
        print(json.dumps(rec), flush=True)

    for row in rows:
        if row in ("rx_c2", "rx_l34_c2", "rx_c3", "rx_u64"):
            wl = {"rx_c3": "c3", "rx_u64": "u64"}.get(row, "c2")
            n, fb, f, d = batch(wl)
            ctx = rss_ctx(16 if wl == "c3" else 4)
            cs = torch.empty(n, dtype=torch.int16, device=dev)
            hs = torch.empty(n, dtype=torch.int32, device=dev)
            qs = torch.empty(n, dtype=torch.int16, device=dev)
            hits = torch.zeros(128, dtype=torch.int64, device=dev)
            l34 = torch.empty(n, dtype=torch.uint8, device=dev) if row == "rx_l34_c2" else None

            def fn():
                sna.rx_offload(ctx, f, d, sna.TUPLE_AUTO, 0, 0, cs, hs, qs, hits, l34=l34)

            region, med = timed(torch, fn, args.steps, args.warmup)
            alg = fb + 16 * n + (n if l34 is not None else 0)
            report(row, wl, n, fb, alg, region, med)
            ctx.close()
        elif row in ("rss_c2", "rss_c3"):
            # hash + queue + hits without checksums: the header-only kernel
            wl = row.split("_")[1]
            n, fb, f, d = batch(wl)
            ctx = rss_ctx(16 if wl == "c3" else 4)
            hs = torch.empty(n, dtype=torch.int32, device=dev)
            qs = torch.empty(n, dtype=torch.int16, device=dev)
            hits = torch.zeros(128, dtype=torch.int64, device=dev)

            def fn():
                sna.rx_offload(ctx, f, d, sna.TUPLE_AUTO, 0, 0, None, hs, qs, hits)

            region, med = timed(torch, fn, args.steps, args.warmup)
            lens = (d.cpu().numpy().view(np.uint64) >> np.uint64(40)).astype(np.int64)
            hdr = int(np.minimum(lens, 48).sum())
            # descriptors + the staged header bytes + hash/queue out
            report(row, wl, n, fb, 16 * n + hdr + 6 * n, region, med, {"header_bytes": hdr})
            ctx.close()
        elif row in ("icrc_c2", "icrc_c3"):
            wl = row.split("_")[1]
            n, fb, f, d = batch(wl)
            crc = torch.empty(n, dtype=torch.int32, device=dev)

            def fn():
                sna.icrc_batch(f, d, sna.ICRC_CALCULATE, crc)

            region, med = timed(torch, fn, args.steps, args.warmup)
            report(row, wl, n, fb, fb + 12 * n, region, med)
        elif row == "tso_c5":
            n, fb, f, d = batch("c5")
            H, MSS = 54, 1448
            nseg = (9000 - H + MSS - 1) // MSS
            hdr = torch.full((n,), H, dtype=torch.int16, device=dev)
            mss = torch.full((n,), MSS, dtype=torch.int16, device=dev)
            base = torch.arange(0, n * nseg, nseg, dtype=torch.int32, device=dev)
            out = torch.empty(n * nseg, dtype=torch.int16, device=dev)

            def fn():
                sna.tso_checksum(f, d, hdr, mss, base, out)

            region, med = timed(torch, fn, args.steps, args.warmup)
            report(row, "c5", n, fb, fb + 16 * n + 2 * n * nseg, region, med, {"segments": n * nseg})
        elif row == "tso_seg_c5":
            n, fb, f, d = batch("c5")
            H, MSS, STRIDE = 54, int(os.environ.get("SEG_MSS", 1448)), int(os.environ.get("SEG_STRIDE", 1536))
            fl_np = np.full(n, sna.SEG_TSO | sna.SEG_VLAN_INSERT | 0x0123, np.uint32)
            cnt, base_np, total = sna.tso_segment_counts(np.full(n, 9000), np.full(n, H), np.full(n, MSS), fl_np)
            hdr = torch.full((n,), H, dtype=torch.int16, device=dev)
            mss = torch.full((n,), MSS, dtype=torch.int16, device=dev)
            base = torch.from_numpy(base_np.view(np.int32)).to(dev)
            fl = torch.from_numpy(fl_np.view(np.int32)).to(dev)
            out = torch.empty(total * STRIDE, dtype=torch.uint8, device=dev)
            ol = torch.empty(total, dtype=torch.int32, device=dev)
            oc = torch.empty(total, dtype=torch.int16, device=dev)

            def fn():
                sna.tso_segment(f, d, hdr, mss, base, fl, out, STRIDE, ol, oc)

            region, med = timed(torch, fn, args.steps, args.warmup)
            written = int(total * (H + 4) + n * (9000 - H))
            # read frames once + write the segments + 8 B desc, 12 B per-frame params, 6 B per segment out
            report(row, "c5", n, fb, fb + written + 20 * n + 6 * total, region, med,
                   {"segments": total, "bytes_written": written})
        elif row == "seg_copy_c5":
            # the segmentation row's ceiling: a plain copy
            # with tso_seg_c5's write pattern (libnicgpu_tune.so
            # nicgpu_tune_seg_copy: each 1506-B segment at the slot stride,
            # its last chunk written in part), best of a small sweep; and the
            # same copy with whole last chunks (pad) for the partial-line cost
            import ctypes

            n, fb, f, d = batch("c5")
            H, MSS, STRIDE = 54, 1448, 1536
            nseg, last = 7, 9000 - 54 - 6 * 1448
            tl = ctypes.CDLL(os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so"))
            vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
            tl.nicgpu_tune_seg_copy.restype = i32
            tl.nicgpu_tune_seg_copy.argtypes = [vp, u32, u32, vp, u32, u32, u32, u32, u32, i32, i32, vp]
            fstride = (9000 + 15) // 16 * 16
            out = torch.empty(n * nseg * STRIDE, dtype=torch.uint8, device=dev)
            sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            written = int(n * nseg * (H + 4) + n * (9000 - H))
            sweep = {}
            for flags in (0, 1, 2, 3):
                for bpc in (4, 8, 16):
                    def fn(flags=flags, bpc=bpc):
                        rc = tl.nicgpu_tune_seg_copy(f.data_ptr(), n, fstride, out.data_ptr(), STRIDE, H + 4, MSS, nseg,
                                                     last, bpc, flags, sp)
                        assert rc == 0, rc
                    sweep[(flags, bpc)] = timed(torch, fn, args.steps, args.warmup)
            best = min((v[1], k) for k, v in sweep.items() if not k[0] & 2)
            best_pad = min((v[1], k) for k, v in sweep.items() if k[0] & 2)
            region = sweep[best[1]][0]
            report(row, "c5", n, fb, fb + written + 20 * n + 6 * n * nseg, region, best[0],
                   {"segments": n * nseg, "bytes_written": written, "best": {"nt": best[1][0] & 1, "blocks_per_cu": best[1][1]},
                    "pad_best_us": round(best_pad[0], 2),
                    "sweep_median_us": {f"nt{k[0] & 1}_pad{k[0] >> 1}_bpc{k[1]}": round(v[1], 2) for k, v in sweep.items()}})
        else:
            raise SystemExit(f"unknown row {row}")


if __name__ == "__main__":
    main()
