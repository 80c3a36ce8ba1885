"""Median per dispatch of every counter of scripts/gpu_pmc_row.sh for kernels
whose name contains the given substring.
  python tools/pmc_row_summary.py gpurun_out/pmc_row tso_segment_kernel"""
import csv
import glob
import statistics
import sys


def main():
    root, pat = sys.argv[1], sys.argv[2]
    vals = {}
    for f in sorted(glob.glob(f"{root}/p*/pmc_counter_collection.csv")):
        per = {}
        for row in csv.DictReader(open(f)):
            if pat not in row["Kernel_Name"]:
                continue
            key = (row["Counter_Name"], row["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        for (c, _), v in per.items():
            vals.setdefault(c, []).append(v)
    for c, v in sorted(vals.items()):
        print(f"{c:24s} {statistics.median(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
