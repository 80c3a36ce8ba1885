"""Batched QueueManager (nic::BatchedQueueManager, SURVEY §8 f1's caller)
against the reference QueueManager drained over several queue pairs
(tests/golden/qm_*.json; oracle/gen_golden.cpp gen_qm_case,
src/queue_manager.cpp:54-78 and :119-139).

cpu: the weighted round-robin schedule (advances, skips, the index/credit a
     round leaves for the next), each run of it through the stage's driver over
     the CPU backend, and the interrupts replayed in the scheduler's order —
     completions, MSI-X vector order, stats and memory bytes as the reference's.
gpu: the product path (every queue's batch on its own device stage, in flight
     at once, when the queues' buffers are disjoint; the reference's
     interleaving on the host path when qm_alias makes the order decide the
     bytes), compared the same way plus QueueManagerStats and stats_summary().
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
