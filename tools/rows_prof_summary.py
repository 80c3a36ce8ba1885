"""Summarise scripts/gpu_rows_prof.sh: for every §8 row, the row's dominant
kernel (largest total time in its rocprofv3 kernel-trace stats), its average
launch duration there, the HIP-event timing bench_rows.py printed in the same
run, and its HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes
(gfx950 correction as tools/pmc_summary.py: read bytes = 2 x FETCH_SIZE x 1024,
written = WRITE_SIZE x 1024) against the row's algorithmic bytes.

  python tools/rows_prof_summary.py gpurun_out/rows_prof TAG > profiles/TAG_rows_prof.json

FETCH_SIZE is calibrated per access shape (profiles/r03_calib_fetch.json,
tools/calib_fetch.py: known-byte kernels of each shape on the same box):
coalesced 16-B/lane streams (RX, TSO, the f1 delivery) and lane-owned 128-B
line walks (ICRC) both count exactly half their bytes (factor 2.0, the guide's
correction, now measured for both shapes).  A sparse header gather (RSS
without checksums: 48 B per frame) has no byte-exact ground truth: the
known-shape kernel reading 48 B at every 1536-B slot shows 147.3 B of
FETCH_SIZE per slot, so those rows report their FETCH_SIZE per packet over
that same-shape minimum instead of a corrected byte count.
"""

import csv
import glob
import json
import os
import statistics
import sys


def top_kernel(stats_csv):
    rows = list(csv.DictReader(open(stats_csv)))
    rows.sort(key=lambda r: float(r["TotalDurationNs"]), reverse=True)
    r = rows[0]
    return r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, [
        {"kernel": x["Name"][:120], "calls": int(x["Calls"]), "avg_us": round(float(x["AverageNs"]) / 1e3, 2)}
        for x in rows[:6]]


def per_dispatch_median(counter_csv, counter, kernel):
    vals = {}
    for r in csv.DictReader(open(counter_csv)):
        if r["Counter_Name"] != counter or r["Kernel_Name"] != kernel:
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return statistics.median(vals.values()) if vals else None


CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r03_calib_fetch.json")
SHAPE = {"rx_c2": "stream", "rx_l34_c2": "stream", "rx_c3": "stream", "rx_u64": "stream", "tso_c5": "stream",
         "tso_seg_c5": "stream", "f1": "stream", "icrc_c2": "linewalk", "icrc_c3": "linewalk",
         "rss_c2": "hdr48", "rss_c3": "hdr48"}


def main():
    root, tag = sys.argv[1], sys.argv[2]
    calib = json.load(open(CALIB))["shapes"]
    out = {"what": "every §8 row's dominant kernel under rocprofv3 (scripts/gpu_rows_prof.sh): kernel-trace "
                   "average beside bench_rows.py's HIP-event timing of the same run, and HBM traffic per launch "
                   "(2 x FETCH_SIZE + WRITE_SIZE, KiB -> B; separate --pmc passes) over the algorithmic bytes",
           "rows": []}
    for d in sorted(glob.glob(os.path.join(root, "kt_*"))):
        row = os.path.basename(d)[3:]
        stats = os.path.join(d, f"{tag}_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        kernel, calls, avg_us, top = top_kernel(stats)
        rec = {"row": row, "kernel": kernel[:160], "calls": calls, "rocprof_avg_us": round(avg_us, 2), "top": top}
        bj = os.path.join(root, f"{row}.json")
        if os.path.exists(bj):
            lines = [json.loads(l) for l in open(bj) if l.startswith("{")]
            if row == "f1" and lines and "frame_GBps" in lines[-1]:
                # the delivery reads and writes every delivered frame once:
                # 2 x the batch's frame bytes (frame_GBps x batch time)
                b = lines[-1]
                rec.update({"stage_batch_us_median": b["us_median"],
                            "alg_bytes_per_launch": int(2 * b["frame_GBps"] * b["us_median"] * 1e3),
                            "alg_bytes_note": "2 x the frames delivered (read + written); write records, statuses and hashes not counted"})
            elif lines and "alg_bytes_per_launch" in lines[0]:
                b = lines[0]
                rec.update({"hip_event_region_us": b.get("us_region_avg"), "hip_event_median_us": b.get("us_median"),
                            "alg_bytes_per_launch": b["alg_bytes_per_launch"]})
        f = os.path.join(root, f"FETCH_SIZE_{row}", f"{tag}_counter_collection.csv")
        w = os.path.join(root, f"WRITE_SIZE_{row}", f"{tag}_counter_collection.csv")
        if os.path.exists(f) and os.path.exists(w):
            fk = per_dispatch_median(f, "FETCH_SIZE", kernel)
            wk = per_dispatch_median(w, "WRITE_SIZE", kernel)
            if fk is not None and wk is not None:
                shape = SHAPE.get(row, "stream")
                c = calib[shape]
                rec.update({"fetch_size_kb": fk, "write_size_kb": wk, "access_shape": shape})
                if "factor" in c:
                    traffic = int(c["factor"] * fk * 1024 + wk * 1024)
                    rec.update({"fetch_factor": c["factor"], "hbm_bytes_per_launch": traffic})
                    if rec.get("alg_bytes_per_launch"):
                        rec["traffic_over_alg"] = round(traffic / rec["alg_bytes_per_launch"], 4)
                else:
                    pk = [json.loads(l) for l in open(bj) if l.startswith("{")][0].get("packets") if os.path.exists(bj) else None
                    if pk:
                        per_pkt = fk * 1024 / pk
                        rec.update({"fetch_bytes_per_packet": round(per_pkt, 2),
                                    "same_shape_min_fetch_bytes_per_slot": c["fetch_bytes_per_slot"],
                                    "fetch_over_same_shape_min": round(per_pkt / c["fetch_bytes_per_slot"], 4)})
                if rec.get("alg_bytes_per_launch"):
                    rec["alg_GBps_rocprof"] = round(rec["alg_bytes_per_launch"] / (avg_us * 1e3), 1)
                    rec["frac_of_8TBps_rocprof"] = round(rec["alg_bytes_per_launch"] / (avg_us * 1e3) / 8000.0, 4)
        out["rows"].append(rec)
    try:
        with open(os.path.join(root, "kernel_source.sha")) as fh:
            out["kernel_source_sha256"] = fh.read().split()[0][:16]
    except OSError:
        pass
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
