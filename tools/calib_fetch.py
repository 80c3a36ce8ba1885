"""FETCH_SIZE calibration per access shape.

MI355X_MICROARCH.md says FETCH_SIZE reports exactly half of the bytes of a
16-B/lane coalesced streaming read on gfx950 and that other access widths are
uncalibrated.  This runs the tuning build's calib_kernel (libnicgpu_tune.so)
once per shape over a 1.5 GB buffer (past the 256 MiB Infinity Cache), each
reading a known set of whole 128-B lines or line prefixes:
  stream     16 B per lane, coalesced (the RX kernel's stream)        true bytes = buffer
  linewalk   lane-owned 128-B lines, 16 B per load (the ICRC kernel)  true bytes = buffer
  hdr48      48 B at every 1536-B slot (rss_only on C2 frames)        true bytes unknown: 64 or 128 per slot
  hdr64      64 B at every 1536-B slot                                 true bytes unknown: 64 or 128 per slot
  hdr128     one whole 128-B line per 1536-B slot                      true bytes = 128 per slot
Run under rocprofv3 --pmc FETCH_SIZE; tools/calib_summary.py divides.
  python tools/calib_fetch.py  (prints the shapes' launch order)"""

import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = ["stream", "linewalk", "hdr48", "hdr64", "hdr128"]


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "smart_nic_amd", "libnicgpu_tune.so"))
    lib.nicgpu_tune_calib.restype = ctypes.c_int
    lib.nicgpu_tune_calib.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    nbytes = 1536 * (1 << 20)  # 1 M slots of 1536 B
    buf = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    order = []
    for rep in range(3):
        for i, name in enumerate(SHAPES):
            rc = lib.nicgpu_tune_calib(i, buf.data_ptr(), nbytes, sink.data_ptr(), s)
            if rc != 0:
                sys.exit(f"calib {name}: {rc}")
            order.append(name)
    torch.cuda.synchronize()
    slots = nbytes // 1536
    print(json.dumps({"order": order, "bytes": nbytes, "slots": slots,
                      "true_bytes": {"stream": nbytes, "linewalk": nbytes, "hdr128": slots * 128}}))


if __name__ == "__main__":
    main()
