"""The hardware assumption under deliver_kernel's edge windows (f1.hip): a
16-B global load or store at any byte alignment is one dwordx4 that moves
exactly those 16 bytes (gfx950 in the HSA unaligned access mode).  The probe
(nicgpu_tune_unaligned_copy, libnicgpu_tune.so) copies 16 B per lane from
every source alignment to every destination alignment, the lanes' windows
overlapping in the source, and the bytes around each destination window stay untouched
(stores are byte-enabled: no read-modify-write of the neighbouring dwords).
GPU only."""

import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("soff,doff", [(0, 0), (1, 3), (2, 2), (3, 1), (14, 7)])
def test_unaligned_16b_copy(soff, doff):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    path = os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so")
    if not os.path.exists(path):
        pytest.fail("libnicgpu_tune.so missing: run __graft_entry__.build()")
    tl = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    tl.nicgpu_tune_unaligned_copy.restype = ctypes.c_int
    tl.nicgpu_tune_unaligned_copy.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp]
    n = 4096
    rng = np.random.default_rng(soff * 31 + doff)
    src = rng.integers(0, 256, 17 * n + 64, dtype=np.uint8)
    fill = rng.integers(0, 256, 19 * n + 64, dtype=np.uint8)
    s_dev = torch.from_numpy(src).cuda()
    d_dev = torch.from_numpy(fill).cuda()
    assert tl.nicgpu_tune_unaligned_copy(s_dev.data_ptr(), d_dev.data_ptr(), n, soff, doff,
                                         torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    want = fill.copy()
    for i in range(n):
        want[19 * i + doff: 19 * i + doff + 16] = src[17 * i + soff: 17 * i + soff + 16]
    got = d_dev.cpu().numpy()
    assert np.array_equal(got, want)
