#!/bin/bash
# Row f1 on C3 (1 M IMIX descriptors, descriptors and results in HBM, pipelined):
# kernel trace of the batch, then FETCH_SIZE / WRITE_SIZE passes (deliver_kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f1prof
cd /tmp && export TMPDIR=/tmp
ARGS="c3 1048576 ${F1_REPS:-6} 0 device device pipelined device"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f1prof/trace -o f1 --output-format csv -- $R/tools/bin/bench_rx_stage $ARGS > $R/gpurun_out/f1prof/trace.log 2>&1 || { tail -5 $R/gpurun_out/f1prof/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/f1prof/fetch -o f1 -- $R/tools/bin/bench_rx_stage $ARGS > $R/gpurun_out/f1prof/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/f1prof/write -o f1 -- $R/tools/bin/bench_rx_stage $ARGS > $R/gpurun_out/f1prof/write.log 2>&1 || { echo write failed; exit 1; }
grep '^{' $R/gpurun_out/f1prof/trace.log | tail -1
python3 - <<'PY'
import csv, glob, statistics
R = __import__("os").environ["GRAFT_REPO_ROOT"] + "/gpurun_out/f1prof"
st = glob.glob(R + "/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(st)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>4}  {r["Name"][:100]}')
for c, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    f = glob.glob(R + f"/{d}/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "deliver_kernel" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    print(c, "deliver_kernel median KB", statistics.median(per.values()), "n", len(per))
PY
