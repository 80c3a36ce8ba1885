"""Batched QueueManager (nic::BatchedQueueManager, SURVEY §8 f1's caller)
against the reference QueueManager drained over several queue pairs
(tests/golden/qm_*.json; oracle/gen_golden.cpp gen_qm_case,
src/queue_manager.cpp:54-78 and :119-139).

cpu: the weighted round-robin schedule (advances, skips, the index/credit a
     round leaves for the next), each run of it through the stage's driver over
     the CPU backend, and the interrupts replayed in the scheduler's order —
     completions, MSI-X vector order, stats and memory bytes as the reference's.
gpu: the product path (every queue pair's batch in ONE fused device batch when
     the queues' buffers are disjoint; the reference's interleaving on the host
     path when qm_alias makes the order decide the bytes), compared the same way
     plus QueueManagerStats and stats_summary().
scale: 16 queue pairs, ~70 K descriptors (tests/golden/qm16_scale.json; the
     input made from its seed by tests/cpp/qm_scale_gen.h on both sides),
     checked by digest on the CPU path, the fused GPU batch and HostMemory.
"""

import json
import os
import subprocess

import pytest

from test_host_cpp import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
CASES = {"qm_mix": True, "qm_weights": True, "qm_alias": False}  # name -> queues disjoint


def _flatten(name, out_dir):
    d = json.load(open(os.path.join(GOLDEN, name + ".json")))
    Q = d["queues"]
    lines = [f'{Q} {d["max_mtu"]} {d["mem_size"]} {len(d["rounds"])}',
             " ".join(str(x) for x in d["weights"]),
             " ".join(str(x) for x in d["enable_tx_interrupts"]),
             " ".join(str(x) for x in d["enable_rx_interrupts"])]
    for r in d["rounds"]:
        lines.append(" ".join(str(x) for x in r["ntx"]))
        lines.append(" ".join(str(x) for x in r["nrx"]))
        lines.append(f'{r["advances"]} {r["skips"]}')
        lines.append(" ".join(str(x) for x in r["rx_consumed"]))
        lines.append(f'{len(r["irq_vectors"])} ' + " ".join(str(x) for x in r["irq_vectors"]))
        for key in ("tx_completions", "rx_completions"):
            for lst in r[key]:
                lines.append(str(len(lst)))
                lines += [" ".join(str(x) for x in c) for c in lst]
    lines += [" ".join(str(x) for x in s) for s in d["stats"]]
    lines.append(" ".join(str(x) for x in d["qm_stats"]))
    lines.append(d["mem_fnv"])
    lines.append(d["stats_summary"])
    path = os.path.join(out_dir, name + ".expect.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def _run(exe, mode, name, tmp_path, extra=()):
    exp = _flatten(name, str(tmp_path))
    args = [exe, mode, exp] + [os.path.join(GOLDEN, f"{name}.{k}.bin") for k in ("mem", "tx", "rx")] + list(extra)
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"qm_test {mode}: ok" in r.stdout


def _flatten_scale(out_dir):
    d = json.load(open(os.path.join(GOLDEN, "qm16_scale.json")))
    Q = d["queues"]
    lines = [f'{Q} {d["max_mtu"]} {d["mem_size"]} {len(d["rounds"])} {d["seed"]}',
             " ".join(str(x) for x in d["weights"])]
    for r in d["rounds"]:
        for key in ("ntx", "nrx"):
            lines.append(" ".join(str(x) for x in r[key]))
        lines.append(f'{r["advances"]} {r["skips"]}')
        lines.append(" ".join(str(x) for x in r["rx_consumed"]))
        lines.append(f'{r["irq_count"]} {r["irq_fnv"]}')
        for key in ("tx_count", "rx_count", "tx_fnv", "rx_fnv"):
            lines.append(" ".join(str(x) for x in r[key]))
    lines += [" ".join(str(x) for x in s) for s in d["stats"]]
    lines.append(" ".join(str(x) for x in d["qm_stats"]))
    lines.append(d["mem_fnv"])
    lines.append(d["stats_summary"])
    path = os.path.join(out_dir, "qm16_scale.expect.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def _run_scale(exe, mode, tmp_path):
    r = subprocess.run([exe, "scale", mode, _flatten_scale(str(tmp_path))], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "qm_test scale: ok" in r.stdout
    print(r.stdout.strip())


def test_scale_fixture_shape():
    """The scale fixture: 16 queue pairs, >= 64 K TX descriptors, an idle queue
    pair the scheduler skips, a ring that runs dry, TSO/GSO segments, checksum
    drops, small buffers and interrupts on most queue pairs."""
    d = json.load(open(os.path.join(GOLDEN, "qm16_scale.json")))
    assert d["queues"] == 16 and sum(sum(r["ntx"]) for r in d["rounds"]) >= 65536
    r0 = d["rounds"][0]
    assert r0["ntx"][5] == 0 and r0["skips"] > 0 and r0["rx_consumed"][7] == r0["nrx"][7]
    qs = d["qm_stats"]  # tx, rx, txb, rxb, drops csum, no_rx, small, tso, gso, vlan ins, strip, verified, gro, adv, skip
    assert qs[4] > 0 and qs[5] > 0 and qs[6] > 0 and qs[7] > 0 and qs[8] > 0 and qs[13] == sum(sum(r["ntx"]) for r in d["rounds"])
    assert all(r["irq_count"] > 0 for r in d["rounds"])


def test_queue_manager_scale_cpu(tmp_path):
    """The CPU path (schedule, run-by-run driver, interrupt replay) reproduces
    the reference QueueManager's digests at 16 queue pairs x 4096."""
    _run_scale(_build(tmp_path, "qm_test"), "cpu", tmp_path)


@pytest.mark.gpu
def test_queue_manager_scale_gpu(tmp_path):
    """The fused device batch at scale, on an HBM image and on FlatHostMemory."""
    exe = _build(tmp_path, "qm_test")
    _run_scale(exe, "gpu", tmp_path)
    _run_scale(exe, "host", tmp_path)


def test_fixture_shape():
    """The fixtures exercise skips, weights above one and zero, rounds that
    carry scheduler state and RX leftovers, and cross-queue aliasing."""
    skips = adv = 0
    weights = set()
    for n in CASES:
        d = json.load(open(os.path.join(GOLDEN, n + ".json")))
        weights |= set(d["weights"])
        assert len(d["rounds"]) == 2
        for r in d["rounds"]:
            skips += r["skips"]
            adv += r["advances"]
            assert r["advances"] == sum(r["ntx"])
        assert d["qm_stats"][13] == sum(r["advances"] for r in d["rounds"])
    assert skips > 0 and adv > 0 and 0 in weights and max(weights) > 2


def test_schedule_counters_only_form(tmp_path):
    """qm_detail::schedule without its runs (whole round-robin cycles counted
    at once, the fused path's form) equals the run-by-run drain."""
    exe = _build(tmp_path, "qm_test")
    r = subprocess.run([exe, "schedule"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "counters-only form equals" in r.stdout


def test_queue_manager_cpu(tmp_path):
    exe = _build(tmp_path, "qm_test")
    for name, disjoint in CASES.items():
        _run(exe, "cpu", name, tmp_path, () if disjoint else ("interleaved",))


@pytest.mark.gpu
def test_queue_manager_gpu(tmp_path):
    exe = _build(tmp_path, "qm_test")
    for name, disjoint in CASES.items():
        _run(exe, "gpu", name, tmp_path, () if disjoint else ("interleaved",))


@pytest.mark.gpu
def test_queue_manager_host_memory_gpu(tmp_path):
    """The same fixtures on a HostMemory (nic::FlatHostMemory): one HBM mirror
    for all queue pairs, the fused batch's TX bytes staged up and its delivered
    bytes written back; the memory's bytes must be the reference's."""
    exe = _build(tmp_path, "qm_test")
    for name, disjoint in CASES.items():
        _run(exe, "host", name, tmp_path, () if disjoint else ("interleaved",))


QM_REFMEM = os.path.join(ROOT, "oracle", "_ref", "qm_test_refmem")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(QM_REFMEM), reason="oracle/_ref/qm_test_refmem not built (make -C oracle ref)")
def test_queue_manager_reference_simple_host_memory_gpu(tmp_path):
    """...and on the reference's own SimpleHostMemory (src/simple_host_memory.cpp
    compiled in place by oracle/Makefile; the binary travels to the GPU box)."""
    for name, disjoint in CASES.items():
        _run(QM_REFMEM, "host", name, tmp_path, () if disjoint else ("interleaved",))
    _run_scale(QM_REFMEM, "host", tmp_path)


@pytest.mark.gpu
def test_queue_manager_fused_fuzz(tmp_path):
    """BatchedQueueManager's fused batch (all queue pairs' batches and rings in
    one device batch, per-queue-pair segments) against each queue pair alone
    through the host resolve, on 60 random managers (1-12 queue pairs, mixed
    MTUs and queue ids, short and empty rings, TSO, VLAN, faults; RSS through a
    shared engine or one per queue pair; results on the host or the device;
    one in three on a HostMemory), two drains each."""
    from test_host_cpp import _build as build
    exe = build(tmp_path, "rx_stage_gpu_fuzz")
    r = subprocess.run([exe, "qm", "60"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rx_stage_gpu_fuzz qm: ok" in r.stdout
    print(r.stdout.strip())
