"""The host side of the drop-in (smart_nic_amd/csrc/host/*.cpp: checksum, RSS,
the batched QueuePair stage's plan/resolve, ICRC) under AddressSanitizer and
UndefinedBehaviorSanitizer — the reference runs its tests under `make asan` in
CI.  CPU paths only; the HIP library is linked unsanitized (GPU
sanitizers are not available on this pool)."""

import os
import subprocess

import pytest

from test_rx_stage import CASES, GOLDEN, _flatten

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "smart_nic_amd")
HOST_SRC = sorted(os.path.join(PKG, "csrc", "host", f) for f in os.listdir(os.path.join(PKG, "csrc", "host"))
                  if f.endswith(".cpp"))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


def _build_san(tmp_path, name):
    if not os.path.exists(os.path.join(PKG, "libnicgpu.so")):
        pytest.fail("smart_nic_amd/libnicgpu.so missing: run __graft_entry__.build()")
    exe = str(tmp_path / f"{name}_san")
    cmd = ["g++", "-std=c++20", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", f"-I{ROOT}/include", f"-I{ROOT}/oracle",
           os.path.join(ROOT, "tests", "cpp", f"{name}.cpp"), *HOST_SRC,
           "-x", "c", os.path.join(ROOT, "oracle", "oracle.c"), "-x", "none",
           f"-L{PKG}", "-lnicgpu", f"-Wl,-rpath,{PKG}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def test_host_api_asan_ubsan(tmp_path):
    exe = _build_san(tmp_path, "host_api_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host_api_test: ok" in r.stdout


def test_icrc_host_asan_ubsan(tmp_path):
    exe = _build_san(tmp_path, "icrc_test")
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "icrc_test cpu: ok" in r.stdout


def test_rx_stage_host_logic_asan_ubsan(tmp_path):
    exe = _build_san(tmp_path, "rx_stage_test")
    for name in CASES:
        exp = _flatten(name, str(tmp_path))
        args = [exe, "cpu", exp] + [os.path.join(GOLDEN, f"{name}.{k}.bin") for k in ("mem", "tx", "rx")]
        r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=ENV)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "rx_stage_test cpu: ok" in r.stdout
