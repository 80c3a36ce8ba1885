"""Summarise tools/calib_fetch.py under rocprofv3 --pmc FETCH_SIZE (and a
second pass of --pmc WRITE_SIZE is not needed: the shapes only read).

  python tools/calib_summary.py <pmc_counter_collection.csv> <calib_fetch stdout json>

For every shape: the median FETCH_SIZE (bytes) per launch, the bytes it must
bring from HBM where they are known, and their ratio — the factor to multiply
FETCH_SIZE by for that access shape (the guide's x2 for coalesced streams)."""

import csv
import json
import statistics
import sys


def main():
    pmc, info = sys.argv[1], json.load(open(sys.argv[2]))
    per = {}
    for r in csv.DictReader(open(pmc)):
        if "calib_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != "FETCH_SIZE":
            continue
        per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    order = info["order"]
    assert len(ids) == len(order), (len(ids), len(order))
    by = {}
    for d, name in zip(ids, order):
        by.setdefault(name, []).append(per[d] * 1024.0)
    out = {"buffer_bytes": info["bytes"], "slots_1536B": info["slots"], "shapes": {}}
    for name, v in by.items():
        med = statistics.median(v)
        e = {"fetch_size_bytes": med, "fetch_bytes_per_slot": round(med / info["slots"], 2)}
        t = info["true_bytes"].get(name)
        if t:
            e["true_bytes"] = t
            e["factor"] = round(t / med, 4)
        out["shapes"][name] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
