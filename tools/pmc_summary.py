"""Summarise the two rocprofv3 PMC passes of scripts/gpu_round.sh into the
per-launch HBM traffic JSON that bench.py reads as `roofline.traffic`.

  python tools/pmc_summary.py gpurun_out/prof TAG > profiles/TAG_pmc_c2.json

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
counts half the bytes of a 16-B/lane coalesced streaming read, so read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is.
"""

import csv
import glob
import json
import statistics
import sys


def per_dispatch(path, counter, kernel_prefix):
    vals = {}
    name = None
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or kernel_prefix not in row["Kernel_Name"]:
            continue
        name = row["Kernel_Name"]
        d = row["Dispatch_Id"]
        vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return name, list(vals.values())


def main():
    root, tag = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "rx_offload_kernel"
    fpath = glob.glob(f"{root}/fetch/{tag}_counter_collection.csv")[0]
    wpath = glob.glob(f"{root}/write/{tag}_counter_collection.csv")[0]
    name, fetch = per_dispatch(fpath, "FETCH_SIZE", kernel)
    _, write = per_dispatch(wpath, "WRITE_SIZE", kernel)
    f_med = statistics.median(fetch)
    w_med = statistics.median(write)
    alg = 1048576 * (1518 + 8 + 8)
    hbm = int(2 * f_med * 1024 + w_med * 1024)
    out = {
        "kernel": name,
        "workload": "C2: 1M x 1518 B TCP, checksum + RSS (bench.py default)",
        "command": "rocprofv3 --pmc FETCH_SIZE (pass 1) / --pmc WRITE_SIZE (pass 2) -- python3 bench.py "
                   "--steps 10 --warmup 2 --no-cpu-baseline --no-e2e (scripts/gpu_round.sh)",
        "fetch_size_kb_median": f_med,
        "write_size_kb_median": w_med,
        "dispatches": len(fetch),
        "correction": "gfx950 FETCH_SIZE counts half the bytes of a 16-B/lane coalesced streaming read "
                      "(MI355X_MICROARCH.md §HBM): read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 as is",
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "ratio_traffic_over_algorithmic": round(hbm / alg, 4),
    }
    # sha256[:16] of the kernel source the GPU run used (scripts/gpu_round.sh writes it)
    try:
        with open(f"{sys.argv[1]}/kernel_source.sha") as f:
            out["kernel_source_sha256"] = f.read().split()[0][:16]
    except OSError:
        pass
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
