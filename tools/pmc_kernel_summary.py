#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (one directory per pass, as
scripts/gpu_r06_o.sh writes them): counters averaged per dispatch for every
kernel whose name contains one of the given substrings, plus the wave-cycle
split (parked on s_waitcnt = SQ_WAIT_ANY, issue-stalled = SQ_WAIT_INST_ANY,
issuing = SQ_ACTIVE_INST_ANY, each over SQ_WAVE_CYCLES) and instructions per
wave.  Tuning aid.

  python tools/pmc_kernel_summary.py gpurun_out/r06o tso_segment_kernel seg_copy_kernel
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    keys = sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [per dispatch]
    for path in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        acc = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            k = next((x for x in keys if x in name), None)
            if k is None:
                continue
            d = (r["Dispatch_Id"], r["Counter_Name"])
            acc[d] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = name
        for (disp, counter), v in acc.items():
            per[names[disp]][counter].append(v)
    out = {}
    for name, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        row = {"dispatches": max(len(v) for v in cs.values()), "avg": {c: round(x, 1) for c, x in avg.items()}}
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
                if c in avg:
                    row.setdefault("frac_of_wave_cycles", {})[c] = round(avg[c] / wc, 4)
        w = avg.get("SQ_WAVES")
        if w:
            row["insts_per_wave"] = {c: round(avg[c] / w, 1) for c in avg if c.startswith("SQ_INSTS_")}
        out[name[:120]] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
