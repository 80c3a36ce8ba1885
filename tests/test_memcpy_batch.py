"""nicgpu_memcpy_batch: the one-launch gather BatchedQueueManager uses to
concatenate the queue pairs' HBM descriptor arrays (include/nicgpu.h).  Plain
byte copies, so the check is the copy itself: every destination range equals
its source, every byte around the ranges keeps its prefill."""

import ctypes

import numpy as np
import pytest

import smart_nic_amd as sna


class CopyRange(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("src", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


def test_memcpy_batch_validates_without_gpu():
    lib = sna.load_library()
    assert lib.nicgpu_memcpy_batch(None, 0, None) == sna.OK
    assert lib.nicgpu_memcpy_batch(None, 1, None) == sna.ERR_INVALID
    r = (CopyRange * 65)()
    assert lib.nicgpu_memcpy_batch(r, 65, None) == sna.ERR_INVALID  # over NICGPU_COPY_BATCH_MAX
    r[0].bytes = 8  # a non-empty range without pointers
    assert lib.nicgpu_memcpy_batch(r, 1, None) == sna.ERR_INVALID


@pytest.mark.gpu
def test_memcpy_batch_gpu():
    import torch

    lib = sna.load_library()
    rng = np.random.default_rng(11)
    # wide (8-B) and byte ranges, empty ones, ragged sizes, 64 at once and a tail launch
    for n in (1, 7, 64):
        sizes = rng.integers(0, 300_000, n)
        sizes[rng.random(n) < 0.2] = 0
        offs_s = rng.integers(0, 64, n)
        offs_d = rng.integers(0, 64, n)
        wide = rng.random(n) < 0.6
        offs_s[wide] &= ~7
        offs_d[wide] &= ~7
        sizes[wide] &= ~7
        total = int((sizes + offs_s + 64).sum())
        src = torch.from_numpy(rng.integers(0, 256, total, dtype=np.uint8)).cuda()
        dst = torch.full((int((sizes + offs_d + 64).sum()),), 0xA5, dtype=torch.uint8, device="cuda")
        r = (CopyRange * n)()
        s_at, d_at, expect = 0, 0, np.full(dst.numel(), 0xA5, np.uint8)
        hsrc = src.cpu().numpy()
        for i in range(n):
            a, b, L = s_at + int(offs_s[i]), d_at + int(offs_d[i]), int(sizes[i])
            r[i].src, r[i].dst, r[i].bytes = src.data_ptr() + a, dst.data_ptr() + b, L
            expect[b:b + L] = hsrc[a:a + L]
            s_at, d_at = a + L + 64 - int(offs_s[i]), b + L + 64 - int(offs_d[i])
        assert lib.nicgpu_memcpy_batch(r, n, None) == sna.OK
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), expect)
