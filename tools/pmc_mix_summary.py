"""Summarise scripts/gpu_pmc_mix.sh: per (workload, mode) the median over the
last 3 rx_offload_kernel dispatches of each counter, plus derived per-tile
instruction counts.  python tools/pmc_mix_summary.py gpurun_out/pmc_mix"""

import csv
import glob
import os
import statistics
import sys

TILES = {"u64": (4 << 20) // 64, "imix": (4 << 20) // 64, "c2": (1 << 20) // 64}


def load(path):
    per = {}
    for row in csv.DictReader(open(path)):
        if "rx_offload_kernel" not in row["Kernel_Name"]:
            continue
        d = int(row["Dispatch_Id"])
        per.setdefault(d, {})
        per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    last = [per[d] for d in sorted(per)[-3:]]
    return {k: statistics.median(x[k] for x in last) for k in last[0]} if last else {}


def main():
    root = sys.argv[1]
    rows = {}
    for d in sorted(glob.glob(os.path.join(root, "*_p[12]"))):
        name = os.path.basename(d)
        wl, mode, _ = name.split("_")
        f = glob.glob(os.path.join(d, "*counter_collection.csv"))
        if f:
            rows.setdefault((wl, mode), {}).update(load(f[0]))
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
            "SQ_WAVES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
            "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_WAIT_INST_LDS"]
    print("%-12s" % "counter" + "".join("%14s" % f"{w}/{m}" for (w, m) in rows))
    for k in keys:
        print("%-22s" % k[3:] + "".join("%14.4g" % r.get(k, float("nan")) for r in rows.values()))
    print("per 64-packet tile:")
    for k in ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD"]:
        print("%-22s" % k[3:] + "".join("%14.1f" % (r.get(k, 0) / TILES[w]) for (w, m), r in rows.items()))
    print("%-22s" % "wave-cyc/tile" + "".join(
        "%14.0f" % (r.get("SQ_WAVE_CYCLES", 0) / TILES[w]) for (w, m), r in rows.items()))
    print("%-22s" % "gui_active us@2.4G" + "".join(
        "%14.1f" % (r.get("GRBM_GUI_ACTIVE", 0) / 2400) for (w, m), r in rows.items()))


if __name__ == "__main__":
    main()
