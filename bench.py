#!/usr/bin/env python3
"""bench.py — device-resident RX checksum + RSS throughput on MI355X.

Metric (BASELINE.json): "Mpkt/s + GB/s device-resident RX checksum+RSS, 1518B
batch; % HBM roofline".  Workload = BASELINE configs[1] (C2): 1 M x 1518 B
Eth/IPv4/TCP frames per GPU (1 % corrupted), checksum verify + RSS with the
40-B Microsoft key and a 128-entry 4-queue table (i % 4), tuple = parsed
IPv4 4-tuple.  One step = one fused nicgpu_rx_offload launch over the whole
resident batch.

Multi-GPU (torchrun): one rank per GPU, each with its own 1 M-packet batch
(weak scaling); the RSS key and table are RCCL-broadcast from rank 0 once
before timing; no collective in the timed loop.

Prints ONE JSON line (rank 0).  See DESIGN.md §5 for the roofline terms.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
PKT_LEN = 1518
N_PER_GPU = 1 << 20
DESC_BYTES = 8
RESULT_BYTES = 8  # u16 csum + u16 queue + u32 hash


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cores():
    """CPUs this process may run on (the box's affinity mask), and the host's count."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    return usable, os.cpu_count() or usable


def cgroup_cpu_limit():
    """The CPU quota of this process's cgroup in CPUs (cgroup v2 cpu.max or v1
    cfs_quota/period), or None when unlimited or unreadable."""
    try:
        with open("/proc/self/cgroup") as f:
            lines = f.read().splitlines()
    except OSError:
        lines = []
    cands = []
    for line in lines:
        parts = line.split(":", 2)
        if len(parts) == 3 and (parts[0] == "0" or "cpu" in parts[1].split(",")):
            rel = parts[2].lstrip("/")
            cands += [os.path.join("/sys/fs/cgroup", rel), os.path.join("/sys/fs/cgroup/cpu", rel)]
    cands += ["/sys/fs/cgroup", "/sys/fs/cgroup/cpu"]
    for d in cands:
        try:
            with open(os.path.join(d, "cpu.max")) as f:
                q, p = f.read().split()[:2]
            if q != "max":
                return float(q) / float(p)
            return None
        except (OSError, ValueError):
            pass
        try:
            with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                q = int(f.read())
            with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                p = int(f.read())
            return q / p if q > 0 else None
        except (OSError, ValueError):
            pass
    return None


def cpu_baseline(frames, desc, table, gpu_out, n_sample_1, label):
    """Reference C++ path (oracle/_ref/libref.so: the reference's own
    src/checksum.cpp + src/rss.cpp, compiled in the build container) or, if it
    is absent, the oracle restatement, timed on this host's cores: one core
    over a bounded sample, then a thread sweep (1, 8, 16, 32, 64, 128 and every
    usable core; one RssEngine per thread, rss.h:43 is not thread-safe) over
    the whole batch.  `value` is the best leg and `cores` the threads that
    produced it; the cgroup quota and the sweep are reported beside it.  Also
    checks the GPU outputs bit-exactly on every leg."""
    from oracle import pyoracle as po

    ref = po.ref_lib()
    kind = "reference" if ref is not None else "port"
    usable, host_cpus = usable_cores()
    quota = cgroup_cpu_limit()
    k = np.frombuffer(MS_KEY, np.uint8)
    t = np.ascontiguousarray(table.astype(np.uint16))
    n_all = desc.size

    def run(n, threads):
        cs = np.zeros(n, np.uint16)
        q = np.zeros(n, np.uint16)
        d = np.ascontiguousarray(desc[:n])
        t0 = time.perf_counter()
        if ref is not None:
            ref.ref_rx_batch(frames.ctypes.data, d.ctypes.data, n, 1, k.ctypes.data, k.size,
                             t.ctypes.data, t.size, cs.ctypes.data, q.ctypes.data, threads)
        else:
            # the restatement is single-threaded; time it on one core
            csum, _, qq, _, _ = po.rx_batch(frames, d, MS_KEY, t)
            cs[:], q[:] = csum, qq
        return time.perf_counter() - t0, cs, q

    dt1, cs1, q1 = run(n_sample_1, 1)
    g_cs, g_q = gpu_out
    ok = bool(np.array_equal(cs1, g_cs[:n_sample_1]) and np.array_equal(q1, g_q[:n_sample_1]))
    sweep = {}
    if ref is not None:
        for threads in sorted({t for t in (1, 8, 16, 32, 64, 128) if t <= usable} | {usable}):
            dt, cs, q = run(n_all, threads) if threads > 1 else (dt1 * n_all / n_sample_1, None, None)
            if cs is not None:
                ok = ok and bool(np.array_equal(cs, g_cs) and np.array_equal(q, g_q))
            sweep[threads] = n_all / dt / 1e6
        cores = max(sweep, key=sweep.get)
        best = sweep[cores]
        n_mt = n_all if cores > 1 else n_sample_1
    else:
        cores, n_mt = 1, n_sample_1
        best = n_sample_1 / dt1 / 1e6
    out = {
        "value": round(best, 4),
        "unit": "Mpkt/s",
        "cores": cores,
        "kind": kind,
        "sample": f"{label}: best leg of a thread sweep, {n_mt} packets on {cores} threads (one RssEngine per "
                  f"thread); 1-thread leg over the first {n_sample_1} packets",
        "value_1core": round(n_sample_1 / dt1 / 1e6, 4),
        "gbs": round(best * 1e6 * float(frames_bytes(desc[:n_mt])) / n_mt / 1e9, 4),
        "gpu_matches_cpu_on_sample": ok,
        "cpu_model": _cpu_model(),
        "usable_cores": usable,
        "host_cpus": host_cpus,
        "cgroup_cpu_quota": (round(quota, 2) if quota is not None else None),
        "effective_cores": (min(usable, int(quota + 0.999)) if quota is not None else usable),
        "thread_sweep_mpkts": {str(t): round(v, 4) for t, v in sweep.items()},
    }
    return out


def frames_bytes(desc):
    return int((desc >> np.uint64(40)).astype(np.int64).sum())


def cpu_rows_baseline(pktgen):
    """The CPU side of the other SURVEY §8 rows, beside the GPU numbers in
    DESIGN.md §5 (bounded samples, this host): C3 IMIX RX through the compiled
    reference (16 threads and 1 core), the reference QueuePair over a C3-style
    batch for row f1 and over C5 TSO frames with every segment materialised
    for row f2 (1 core; the reference is single-threaded), and — the
    reference TUs for these are not buildable here or have no batch entry
    point — the oracle restatement on one core for the C5 TSO segment
    checksums, the L3/L4 verification (row f3) and the C2 ICRC."""
    import ctypes

    from oracle import pyoracle as po

    vp = ctypes.c_void_p
    rows = []
    ref = po.ref_lib()
    cores = usable_cores()[0]
    n3 = 1 << 20
    lens = pktgen.imix_lengths(n3, np.random.default_rng(33))
    f3, d3, _ = pktgen.make_batch(lens, seed=33, proto=17, corrupt_frac=0.01)
    k = np.frombuffer(MS_KEY, np.uint8)
    t16 = (np.arange(128) % 16).astype(np.uint16)
    cs = np.zeros(n3, np.uint16)
    q = np.zeros(n3, np.uint16)
    if ref is not None:
        def rx(n, threads):
            t0 = time.perf_counter()
            ref.ref_rx_batch(f3.ctypes.data, d3.ctypes.data, n, 1, k.ctypes.data, k.size, t16.ctypes.data, t16.size,
                             cs.ctypes.data, q.ctypes.data, threads)
            return time.perf_counter() - t0
        sweep = {t: n3 / rx(n3, t) / 1e6 for t in sorted({min(16, cores), min(64, cores), cores})}
        best_t = max(sweep, key=sweep.get)
        dt1 = rx(1 << 16, 1)
        rows.append({"row": "rx_c3", "value": round(sweep[best_t], 4), "unit": "Mpkt/s", "cores": best_t,
                     "kind": "reference", "value_1core": round((1 << 16) / dt1 / 1e6, 4),
                     "thread_sweep_mpkts": {str(t): round(v, 4) for t, v in sweep.items()},
                     "sample": f"{n3} IMIX frames (7:4:1 64/576/1518 B), 16 queues, best of a thread sweep; "
                               f"1 core over 65536"})
    L = po.lib()
    n5 = 4096
    f5, d5, _ = pktgen.make_batch(np.full(n5, 9000), seed=55, proto=6, corrupt_frac=0.0)
    h = np.full(n5, 54, np.uint16)
    m = np.full(n5, 1448, np.uint16)
    out = np.zeros(n5 * 64, np.uint16)
    t0 = time.perf_counter()
    nseg = L.oracle_tso_checksum_batch(vp(f5.ctypes.data), vp(d5.ctypes.data), n5, vp(h.ctypes.data),
                                       vp(m.ctypes.data), vp(out.ctypes.data))
    dt = time.perf_counter() - t0
    rows.append({"row": "tso_c5", "value": round(n5 / dt / 1e6, 4), "unit": "Mpkt/s", "cores": 1, "kind": "port",
                 "gbs": round(n5 * 9000 / dt / 1e9, 4),
                 "sample": f"{n5} x 9000 B frames, H 54, mss 1448 ({nseg} segment checksums)"})
    # row f1: the reference's own QueuePair::process_once over a C3-style
    # batch (oracle/_ref/ref_qp_bench, compiled from the reference sources in
    # the build container; the GPU side is tools/bench_rx_stage.cpp)
    qp_bench = os.path.join(ROOT, "oracle", "_ref", "ref_qp_bench")
    if os.path.exists(qp_bench):
        import json as _json
        import subprocess

        # row f1 (C3 descriptors, C5 TSO with RX verify), then row f2's
        # materialised segmentation: the same QueuePair building and writing
        # every TSO segment of C5
        for args in ([str(1 << 18), "3", "c3"], [str(1 << 15), "3", "c5"], [str(1 << 14), "3", "c5seg"]):
            r = subprocess.run([qp_bench, *args], capture_output=True, text=True, timeout=120)
            if r.returncode == 0 and r.stdout.strip():
                rows.append(_json.loads(r.stdout.strip().splitlines()[-1]))
    # row f3: the L3/L4 verification of the restatement (the reference has no
    # RX-side L3/L4 verify; PacketGenerator's checksums are its definition)
    n34 = 1 << 15
    f34, d34, _ = pktgen.make_batch(np.full(n34, 1518), seed=42, proto=6, corrupt_frac=0.0)
    fl = np.zeros(n34, np.uint8)
    t0 = time.perf_counter()
    L.oracle_l34_batch(vp(f34.ctypes.data), vp(d34.ctypes.data), n34, vp(fl.ctypes.data))
    dt = time.perf_counter() - t0
    rows.append({"row": "l34_c2", "value": round(n34 / dt / 1e6, 4), "unit": "Mpkt/s", "cores": 1, "kind": "port",
                 "gbs": round(n34 * 1518 / dt / 1e9, 4),
                 "sample": f"{n34} x 1518 B TCP frames, IPv4 header + TCP pseudo-header checksum verification"})
    n2 = 1 << 15
    f2, d2, _ = pktgen.make_batch(np.full(n2, 1518), seed=42, proto=6, corrupt_frac=0.0)
    crc = np.zeros(n2, np.uint32)
    t0 = time.perf_counter()
    L.oracle_icrc_batch(vp(f2.ctypes.data), vp(d2.ctypes.data), n2, vp(crc.ctypes.data))
    dt = time.perf_counter() - t0
    rows.append({"row": "icrc_c2", "value": round(n2 / dt / 1e6, 4), "unit": "Mpkt/s", "cores": 1, "kind": "port",
                 "gbs": round(n2 * 1518 / dt / 1e9, 4), "sample": f"{n2} x 1518 B spans, CRC-32C"})
    return rows


def gpu_rows():
    """Every other SURVEY §8 row measured live on this box, after the timed
    region (child processes, one at a time): the RX kernel on C3 IMIX and
    64 B, L3/L4 verification, ICRC, TSO checksums and segmentation
    (tools/bench_rows.py: HIP events per launch, medians, algorithmic bytes
    and roofline fraction per row), RSS without checksums, and the batched
    QueuePair stage of row f1 on C3 and C5, one batch at a time and pipelined,
    with host and with device-resident descriptors and results, on the
    reference's HostMemory (host bytes staged to an HBM mirror and written
    back), with interrupt callbacks, and BatchedQueueManager over 16 queue
    pairs as one fused batch
    (tools/bin/bench_rx_stage, built by __graft_entry__.build()).  Errors are
    reported, never hidden."""
    import subprocess

    rows, errors = [], []
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_rows.py"), "--steps", "10", "--warmup", "2",
                            "--rows", "rx_c3,rx_u64,rx_l34_c2,rss_c2,rss_c3,icrc_c2,icrc_c3,tso_c5,tso_seg_c5"],
                           capture_output=True, text=True, timeout=300)
        rows += [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
        if r.returncode != 0:
            errors.append(f"bench_rows.py rc={r.returncode}: {r.stderr[-400:]}")
    except Exception as e:  # report, never hide
        errors.append(f"bench_rows.py: {e!r}")
    stage = os.path.join(ROOT, "tools", "bin", "bench_rx_stage")
    for args in (["c3", "1048576", "6", "0", "device", "pinned", "sync"],
                 ["c3", "1048576", "12", "0", "device", "pinned", "pipelined"],
                 ["c5", "131072", "6", "0", "device", "pinned", "sync"],
                 # descriptor rings and results kept in HBM (DeviceDescriptors, results_on_device)
                 ["c3", "1048576", "6", "0", "device", "device", "sync", "device"],
                 ["c3", "1048576", "12", "0", "device", "device", "pipelined", "device"],
                 # TX and RX interrupt callbacks on (2 M per batch, replayed in posting order)
                 ["c3", "1048576", "6", "0", "device", "device", "pipelined", "device", "irq"],
                 # the reference's HostMemory interface: TX bytes staged into an HBM
                 # mirror, delivered bytes written back over PCIe (FlatHostMemory)
                 ["c3", "1048576", "8", "0", "device", "hostmem", "pipelined"],
                 # the same with the results kept in HBM (no 38 MB of pageable result
                 # downloads sharing the link with the write-backs: profiles/r06_hostmem_ab.txt)
                 ["c3", "1048576", "8", "0", "device", "hostmem", "pipelined", "device"],
                 # nic::BatchedQueueManager: 16 queue pairs x 64 K C3 descriptors, one
                 # drain as one fused device batch; host, HBM and HostMemory descriptors
                 ["qm16", "1048576", "6", "0", "device", "pinned", "sync", "device"],
                 ["qm16", "1048576", "6", "0", "device", "device", "sync", "device"],
                 ["qm16", "1048576", "4", "0", "device", "hostmem", "sync", "device"]):
        try:
            r = subprocess.run([stage, *args], capture_output=True, text=True, timeout=180)
            rows += [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
            if r.returncode != 0:
                errors.append(f"bench_rx_stage {' '.join(args)} rc={r.returncode}: {r.stderr[-400:]}")
        except Exception as e:
            errors.append(f"bench_rx_stage {' '.join(args)}: {e!r}")
    return rows, errors


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(path):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (see
    profiles/README.md) and where it came from: the profile names the kernel
    source it measured (tools/kernel_sha.py "rx": the RX kernel's sources); a profile
    of another source is reported as stale, never silently."""

    try:
        with open(path) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None, {"profile": os.path.relpath(path, ROOT), "error": "unreadable"}
    from tools.kernel_sha import kernel_source_sha

    cur = kernel_source_sha("rx")
    cur = cur[:16] if cur else None
    rec = prof.get("kernel_source_sha256")
    info = {"profile": os.path.relpath(path, ROOT), "measured_in_this_run": False,
            "profile_kernel_source": rec, "current_kernel_source": cur,
            "stale": (rec is None or rec != cur)}
    if info["stale"]:
        log(f"warning: {info['profile']} was measured on kernel source {rec}, this tree is {cur}: traffic may be stale")
    return prof.get("hbm_bytes_per_launch"), info


def load_rows_traffic(path):
    """Per-row HBM traffic from a committed rows profile (tools/rows_prof_summary.py:
    FETCH_SIZE calibrated per access shape), with the kernel source it measured;
    a profile of another source is reported as stale, never silently."""

    try:
        with open(path) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return {"profile": os.path.relpath(path, ROOT), "error": "unreadable"}
    from tools.kernel_sha import kernel_source_sha

    cur = kernel_source_sha("all")
    cur = cur[:16] if cur else None
    rec = prof.get("kernel_source_sha256")
    keep = ("rocprof_avg_us", "access_shape", "fetch_factor", "hbm_bytes_per_launch", "traffic_over_alg",
            "fetch_bytes_per_packet", "fetch_over_same_shape_min", "frac_of_8TBps_rocprof")
    rows = {r["row"]: {k: r[k] for k in keep if k in r} for r in prof.get("rows", [])}
    return {"profile": os.path.relpath(path, ROOT), "measured_in_this_run": False, "profile_kernel_source": rec,
            "current_kernel_source": cur, "stale": rec is None or rec != cur, "rows": rows}


METRIC_TEXT = {
    "c2": "Mpkt/s + GB/s device-resident RX checksum+RSS, 1518B batch; % HBM roofline",
    "c3": "Mpkt/s + GB/s device-resident RX checksum+RSS, IMIX batch; % HBM roofline",
}

WORKLOAD_TEXT = {
    "c2": "C2: 1M x 1518 B TCP per GPU, checksum verify + RSS (MS 40-B key, 128-entry table i%4, IPv4 4-tuple)",
    "c3": "C3: IMIX 64/576/1518 B at 7:4:1, 4M packets per GPU (job batch byte-sharded), checksum verify + RSS "
          "(MS 40-B key, 128-entry table i%16, IPv4 4-tuple)",
}


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`bench.py --gpus N` (N > 1) started without a launcher: run the same
    command as N rank processes under a torch.distributed.run CHILD process
    (one process per GPU, LOCAL_RANK = GPU index, RCCL over xGMI; gloo for
    --dry-run) and exit with its status.  Nothing here touches the GPU: the
    process is never exec'd into another one and device_count() does not
    initialise HIP on this image.  Rank 0 prints the one JSON line to the
    inherited stdout; a failing rank makes torch.distributed.run stop the
    others and return non-zero, which this process returns."""
    import subprocess

    if not args.dry_run:
        import torch

        have = torch.cuda.device_count()
        if have < args.gpus:
            log(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) are visible")
            return 2
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    log(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def dry_run(args):
    """The multi-rank path without a GPU (gloo on the CPU): rank setup, the
    shard plan, the key/table broadcast from rank 0 (the other ranks start
    from zeros), barriers around an empty timed loop, the max over ranks and
    the job-wide queue_hits reduction, then rank 0's line with n_gpus = world.
    No packet is processed (the step is empty, so `value` is null): it exists
    so a CPU test can run the launcher end to end (tests/test_bench_launch.py)."""
    import hashlib

    import torch

    from smart_nic_amd import dist as sdist

    if "WORLD_SIZE" not in os.environ:  # --gpus 1 --dry-run: a one-rank group
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    ranks = sdist.init_ranks(force=True, backend="gloo")
    rank, world = ranks.rank, ranks.world
    shard = sdist.plan_shard(args.workload, ranks, args.packets)
    table = (np.arange(128) % shard.queues).astype(np.uint16)
    key_t, tab_t = sdist.setup_rss(ranks, MS_KEY if rank == 0 else bytes(len(MS_KEY)),
                                   table if rank == 0 else np.zeros_like(table))
    got = hashlib.sha256(bytes(key_t.numpy()) + tab_t.numpy().tobytes()).hexdigest()[:16]
    want = hashlib.sha256(MS_KEY + table.astype(np.int16).tobytes()).hexdigest()[:16]
    sdist.barrier(ranks)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    sdist.barrier(ranks)
    t_max = sdist.max_over_ranks(time.perf_counter() - t0, ranks.dist)
    per = sdist.gather_over_ranks([shard.hi - shard.lo, got == want], ranks.dist)
    hits = torch.zeros(128, dtype=torch.int64)
    job_hits, _, hits_ok = sdist.job_queue_hits(ranks, hits)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC_TEXT[args.workload], "value": None, "unit": "Mpkt/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_max / max(args.steps, 1) * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "dry run (gloo, no GPU, no packets processed)", "dry_run": True,
            "config": {"workload": WORKLOAD_TEXT[args.workload], "job_packets": shard.job_packets,
                       "parallelism": f"replicas x{world} (gloo dry run)"},
            "per_rank": [{"rank": r, "packets": int(p[0]), "rss_config_broadcast_ok": bool(p[1])}
                         for r, p in enumerate(per)],
            "rss_config_sha": got, "job_queue_hits_ok": bool(hits_ok and int(job_hits.sum()) == 0),
        }), flush=True)
    sdist.finish(ranks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("c2", "c3"), default="c2",
                    help="c2 (BASELINE configs[1], the metric's config) or c3 (IMIX, byte-balanced shards)")
    ap.add_argument("--packets", type=int, default=None, help="packets per GPU (default: the workload's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the same-box read-only streaming ceiling")
    ap.add_argument("--no-rows", action="store_true",
                    help="skip the other SURVEY §8 rows (tools/bench_rows.py and the f1 stage, ~2 min) at N = 1")
    ap.add_argument("--dist", action="store_true",
                    help="take the multi-rank path (RCCL init, key/table broadcast, barriers, max-reduce) even at "
                         "world size 1, to exercise it on a one-GPU box")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06w_pmc_c2.json"))
    ap.add_argument("--rows-prof-json", default=os.path.join(ROOT, "profiles", "r06x_rows_prof.json"))
    ap.add_argument("--dry-run", action="store_true",
                    help="run the rank machinery on gloo/CPU without a GPU or packets (launcher test)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher around us: start the N ranks ourselves (child process)
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        log(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}: refusing to report a mislabelled run")
        sys.exit(2)
    if args.dry_run:
        dry_run(args)
        return

    import torch

    import smart_nic_amd as sna
    from smart_nic_amd import dist as sdist
    from smart_nic_amd import pktgen

    ranks = sdist.init_ranks(force=args.dist, backend="nccl")
    rank, world, dev = ranks.rank, ranks.world, ranks.device
    shard = sdist.plan_shard(args.workload, ranks, args.packets)

    n = shard.lengths.size
    t0 = time.time()
    frames, desc, corrupted = pktgen.make_batch(shard.lengths, seed=shard.seed, proto=shard.proto, corrupt_frac=0.01)
    bytes_local = int(shard.lengths.sum())
    log(f"[rank {rank}] {args.workload}: packets [{shard.lo}, {shard.hi}) of {shard.job_packets}, "
        f"{bytes_local / 1e9:.2f} GB in {time.time() - t0:.1f}s")
    table = (np.arange(128) % shard.queues).astype(np.uint16)

    f_dev = torch.from_numpy(frames).to(dev)
    d_dev = torch.from_numpy(desc.view(np.int64)).to(dev)
    cs = torch.empty(n, dtype=torch.int16, device=dev)
    hs = torch.empty(n, dtype=torch.int32, device=dev)
    qs = torch.empty(n, dtype=torch.int16, device=dev)
    hits = torch.zeros(128, dtype=torch.int64, device=dev)

    # RSS key + table: rank 0's copy, RCCL-broadcast over xGMI to every rank.
    key_dev, tab_dev = sdist.setup_rss(ranks, MS_KEY, table)
    ctx = sna.RssContext(dev.index)
    ctx.set_key_device(key_dev)
    ctx.set_table_device(tab_dev)
    torch.cuda.synchronize()

    def step():
        sna.rx_offload(ctx, f_dev, d_dev, sna.TUPLE_AUTO, 0, 0, cs, hs, qs, hits)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # One HIP event pair on the launch stream (torch's current stream) around
    # the K launches: average launch duration = region / K, inter-launch gaps
    # included. Per-launch event pairs inside the timed loop cost ~8 us of wall
    # time per step on MI355X (tools/launch_gap.py: 259 -> 251 us per C2 step),
    # so the per-launch spread is taken in a separate, untimed pass below.
    stream = torch.cuda.current_stream()
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sdist.barrier(ranks)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ev_a.record(stream)
    for i in range(args.steps):
        step()
    ev_b.record(stream)
    torch.cuda.synchronize()
    sdist.barrier(ranks)
    t_wall = time.perf_counter() - t_start
    kern_avg_s = ev_a.elapsed_time(ev_b) / 1e3 / args.steps

    # untimed: per-launch event pairs for the median launch duration
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(min(args.steps, 20))]
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    kern_med_s = float(np.median([a.elapsed_time(b) for a, b in ev])) / 1e3

    ceiling = read_ceiling(torch, f_dev) if (rank == 0 and world == 1 and not args.no_ceiling) else None

    t_max = sdist.max_over_ranks(t_wall, ranks.dist, dev)
    # per-rank [local GPU index, packets, wall s, kernel avg s, kernel median s]
    per_rank = sdist.gather_over_ranks([ranks.local, n, t_wall, kern_avg_s, kern_med_s], ranks.dist, dev)

    # one more launch with the histogram zeroed: the job-wide RssStats of one
    # batch (all-reduce of the per-table-index hits), checked against the
    # per-rank histograms and against this rank's hashes
    hits.zero_()
    step()
    torch.cuda.synchronize()
    job_hits, per_rank_hits, hits_sum_ok = sdist.job_queue_hits(ranks, hits)

    # correctness of this run (cheap properties on every rank)
    g_cs = cs.cpu().numpy().view(np.uint16)
    g_h = hs.cpu().numpy().view(np.uint32)
    g_q = qs.cpu().numpy().view(np.uint16)
    status_ok = bool(np.array_equal(g_cs != 0, corrupted))
    queue_ok = bool(np.array_equal(g_q, table[g_h % 128]))
    local_hits_ok = bool(np.array_equal(per_rank_hits[rank], np.bincount(g_h % 128, minlength=128).astype(np.uint64)))
    checks = {"status_matches_corruption": status_ok, "queue_is_table_of_hash": queue_ok,
              "queue_hits_is_bincount_of_table_index": local_hits_ok}
    checks_all = sdist.sum_over_ranks(int(all(checks.values())), ranks.dist, dev)
    job_hits_ok = bool(hits_sum_ok and int(job_hits.sum()) == shard.job_packets)

    total_pkts = shard.job_packets * args.steps
    value = total_pkts / t_max / 1e6
    alg_bytes = bytes_local + n * (DESC_BYTES + RESULT_BYTES)
    achieved_gbs = alg_bytes / kern_avg_s / 1e9
    frame_gbs = bytes_local / kern_avg_s / 1e9

    out = None
    if rank == 0:
        traffic, traffic_src = load_traffic(args.traffic_json) if args.workload == "c2" else (None, None)
        out = {
            "metric": METRIC_TEXT[args.workload],
            "value": round(value, 3),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded Eth/IPv4/" + ("TCP" if shard.proto == 6 else "UDP") +
                    " frames, valid IPv4+L4 checksums, whole-frame balancing word, 1% corrupted)",
            "config": {
                "workload": WORKLOAD_TEXT[args.workload],
                "packets_per_gpu": n,
                "job_packets": shard.job_packets,
                "job_bytes": shard.job_bytes,
                "packet_bytes": PKT_LEN if args.workload == "c2" else "imix",
                "parallelism": f"replicas x{world} (contiguous packet shards"
                               + (", byte-balanced" if args.workload == "c3" else "")
                               + ", key/table RCCL broadcast, no data-path collective)",
            },
            "gbs_frames": round(shard.job_bytes / kern_avg_s / 1e9, 2) if world > 1 else round(frame_gbs, 2),
            "gbs_frames_per_gpu": round(frame_gbs, 2),
            "kernel_us_avg": round(kern_avg_s * 1e6, 2),
            "kernel_us_median": round(kern_med_s * 1e6, 2),
            "kernel_timing": "kernel_us_avg = one HIP event pair around the K timed launches / K (gaps included); "
                             "kernel_us_median from per-launch event pairs in a separate untimed pass",
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": alg_bytes,
                "ceiling_measured": ceiling,
                "frac_of_ceiling": (round(achieved_gbs / ceiling["gbs"], 4) if ceiling else None),
            },
            "per_rank": [{"rank": r, "gpu": int(p[0]), "packets": int(p[1]), "ms_per_step": round(p[2] / args.steps * 1e3, 4),
                          "kernel_us_avg": round(p[3] * 1e6, 2), "kernel_us_median": round(p[4] * 1e6, 2)}
                         for r, p in enumerate(per_rank)],
            "kernel_us_avg_max_over_ranks": round(max(p[3] for p in per_rank) * 1e6, 2),
            "checks": dict(checks, all_ranks_ok=checks_all == world, job_queue_hits_ok=job_hits_ok),
            "rss_stats_job": {"hashes": int(job_hits.sum()), "queue_hits_nonzero": int((job_hits > 0).sum()),
                              "queue_hits_per_rank_sum": [int(h.sum()) for h in per_rank_hits]},
        }
    # end-to-end (host pinned -> H2D -> kernel -> D2H of results) and the CPU
    # baseline: rank 0 at N = 1 only
    if rank == 0 and world == 1 and not args.no_e2e and args.workload == "c2":
        try:
            out["e2e"] = e2e_rate(torch, sna, ctx, frames, desc, dev)
        except Exception as e:  # report, never hide
            out["e2e"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_rows:
        out["gpu_rows"], errors = gpu_rows()
        if errors:
            out["gpu_rows_errors"] = errors
        out["gpu_rows_traffic"] = load_rows_traffic(args.rows_prof_json)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(frames, desc, table, (g_cs, g_q), n_sample_1=min(n, 1 << 16),
                                           label=args.workload.upper())
        out["cpu_baseline"]["other_rows"] = cpu_rows_baseline(pktgen)
    if rank == 0:
        print(json.dumps(out), flush=True)
    sdist.finish(ranks)


def read_ceiling(torch, buf, reps=5):
    """Same-box read-only streaming ceiling: the best of a few
    grid shapes of the tuning build's plain 16-B-per-lane streaming read
    kernel over the resident frame buffer, HIP events per launch, median of
    `reps`. Reported beside the 8 TB/s spec peak; never used as `peak`."""
    import ctypes

    path = os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so")
    if not os.path.exists(path):
        return None
    tl = ctypes.CDLL(path)
    vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    tl.nicgpu_tune_stream_read.restype = i32
    tl.nicgpu_tune_stream_read.argtypes = [vp, sz, i32, i32, vp, vp]
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    nbytes = buf.numel() // 16 * 16
    sink = torch.zeros(1, dtype=torch.int32, device=buf.device)
    best = None
    for unroll, bpc in ((1, 8), (2, 4), (4, 2), (4, 4), (8, 2)):
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            rc = tl.nicgpu_tune_stream_read(buf.data_ptr(), nbytes, bpc, unroll, sink.data_ptr(), sp)
            b.record(stream)
            torch.cuda.synchronize()
            if rc != 0:
                return None
            ts.append(a.elapsed_time(b) * 1e3)
        gbs = nbytes / float(np.median(ts)) / 1e3
        if best is None or gbs > best["gbs"]:
            best = {"gbs": round(gbs, 1), "unroll": unroll, "blocks_per_cu": bpc, "bytes": nbytes,
                    "kernel": "stream_read_kernel (libnicgpu_tune.so), same buffer, median of %d" % reps}
    return best


def e2e_rate(torch, sna, ctx, frames, desc, dev, chunk_pkts=1 << 16, reps=3):
    """Packets from pinned host memory through H2D copy, the kernel and D2H of
    the results, chunked and double-buffered over two streams."""
    n = desc.size
    h_frames = torch.from_numpy(frames).pin_memory()
    slot = PKT_LEN + (-PKT_LEN) % 16
    nch = (n + chunk_pkts - 1) // chunk_pkts
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    bufs = []
    for s in range(2):
        bufs.append({
            "f": torch.empty(chunk_pkts * slot + 64, dtype=torch.uint8, device=dev),
            "d": torch.empty(chunk_pkts, dtype=torch.int64, device=dev),
            "cs": torch.empty(chunk_pkts, dtype=torch.int16, device=dev),
            "q": torch.empty(chunk_pkts, dtype=torch.int16, device=dev),
            "h": torch.empty(chunk_pkts, dtype=torch.int32, device=dev),
        })
    # per-chunk descriptors rebased to the chunk buffer
    d_local = desc.copy()
    offs = (desc & np.uint64((1 << 40) - 1)).astype(np.int64)
    h_desc = []
    for c in range(nch):
        a, b = c * chunk_pkts, min(n, (c + 1) * chunk_pkts)
        base = offs[a]
        dd = d_local[a:b] - np.uint64(base)
        h_desc.append(torch.from_numpy(dd.view(np.int64)).pin_memory())
    h_cs = torch.empty(n, dtype=torch.int16).pin_memory()
    h_q = torch.empty(n, dtype=torch.int16).pin_memory()
    h_h = torch.empty(n, dtype=torch.int32).pin_memory()
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c in range(nch):
            s = streams[c % 2]
            B = bufs[c % 2]
            a, b = c * chunk_pkts, min(n, (c + 1) * chunk_pkts)
            fa, fb = int(offs[a]), int(offs[b - 1]) + slot
            with torch.cuda.stream(s):
                B["f"][: fb - fa].copy_(h_frames[fa:fb], non_blocking=True)
                B["d"][: b - a].copy_(h_desc[c], non_blocking=True)
                sna.rx_offload(ctx, B["f"], B["d"][: b - a], sna.TUPLE_AUTO, 0, 0,
                               B["cs"], B["h"], B["q"], None, stream=s)
                h_cs[a:b].copy_(B["cs"][: b - a], non_blocking=True)
                h_q[a:b].copy_(B["q"][: b - a], non_blocking=True)
                h_h[a:b].copy_(B["h"][: b - a], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return {"mpkts": round(n / best / 1e6, 2), "gbs_frames": round(n * PKT_LEN / best / 1e9, 2),
            "chunk_packets": chunk_pkts, "streams": 2,
            "note": "pinned host frames -> H2D -> kernel -> D2H(csum,queue,hash); PCIe-bound"}


if __name__ == "__main__":
    main()
