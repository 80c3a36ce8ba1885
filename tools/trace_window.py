"""Print one batch window of a rocprofv3 trace (tuning aid):
python tools/trace_window.py <kernel_trace.csv> <anchor kernel substring> [k-th from last]

With a memory_copy_trace.csv beside the kernel trace (rocprofv3
--memory-copy-trace), the copies that overlap the window are listed too
(H2D/D2H, bytes when the trace has them), so a timeline shows uploads and
write-backs in flight beside the kernels."""
import csv
import glob
import os
import sys


def main():
    rows = [dict(r, _kind="K") for r in csv.DictReader(open(sys.argv[1]))]
    d = os.path.dirname(sys.argv[1])
    copies = []
    for path in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        copies = [dict(r, _kind="C") for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    anchor = sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    a, b = idx[-k], idx[-k + 1]
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["End_Timestamp"])
    window = rows[a:b + 1]
    for c in copies:
        s, e = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
        if e >= t0 and s <= t1:
            window.append(c)
    window.sort(key=lambda r: int(r["Start_Timestamp"]))
    for r in window:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        if r["_kind"] == "K":
            what = f"q{r['Queue_Id']} {r['Kernel_Name'][:80]}"
        else:
            size = r.get("Bytes") or r.get("Size") or ""
            what = f"copy {r.get('Direction', '')} {size}"
        print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f} {what}")


if __name__ == "__main__":
    main()
