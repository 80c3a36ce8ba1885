"""Build and run the C++ tests of the drop-in nic:: API (libnic_host.so).

host_api_test  — CPU only: checksum/RSS semantics vs the reference's own test
                 expectations and the oracle.
gpu_batch_test — GPU batch entry points vs the per-packet API (marker gpu).
Both link libnic_host.so -> libnicgpu.so through the C-ABI only.
"""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "smart_nic_amd")
INC = os.path.join(ROOT, "include")
ORACLE = os.path.join(ROOT, "oracle")


def _build(tmp_path, name):
    src = os.path.join(ROOT, "tests", "cpp", f"{name}.cpp")
    exe = str(tmp_path / name)
    host_lib = os.path.join(PKG, "libnic_host.so")
    if not os.path.exists(host_lib):
        pytest.fail("smart_nic_amd/libnic_host.so missing: run __graft_entry__.build()")
    # oracle.c is C: compile it as C with an explicit language switch
    cmd = ["g++", "-std=c++20", "-O2", f"-I{INC}", f"-I{ORACLE}", src, "-x", "c", os.path.join(ORACLE, "oracle.c"),
           "-x", "none", f"-L{PKG}", "-lnic_host", "-lnicgpu", f"-Wl,-rpath,{PKG}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_host_api_cpu(tmp_path):
    exe = _build(tmp_path, "host_api_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_api_test: ok" in r.stdout


@pytest.mark.gpu
def test_gpu_batch_api(tmp_path):
    exe = _build(tmp_path, "gpu_batch_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu_batch_test: ok" in r.stdout


def test_icrc_host_cpu(tmp_path):
    exe = _build(tmp_path, "icrc_test")
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "icrc_test cpu: ok" in r.stdout


@pytest.mark.gpu
def test_icrc_batch_gpu(tmp_path):
    exe = _build(tmp_path, "icrc_test")
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "icrc_test gpu: ok" in r.stdout
