#!/bin/bash
# deliver_kernel instruction mix and stall counters (two --pmc passes, kernel trace off)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f1pmc
cd /tmp && export TMPDIR=/tmp
ARGS="c3 1048576 4 0 device device sync device"
P1="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/f1pmc/p$i -o f1 -- $R/tools/bin/bench_rx_stage $ARGS > $R/gpurun_out/f1pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/f1pmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, statistics
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/f1pmc"
for i in (1, 2):
    f = glob.glob(f"{R}/p{i}/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        for k in ("deliver_kernel", "rx_offload_kernel", "qp_full_kernel"):
            if k in r["Kernel_Name"]:
                per.setdefault((k, r["Counter_Name"]), {}).setdefault(r["Dispatch_Id"], 0.0)
                per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for (k, c), v in sorted(per.items()):
        print(f"{k:18s} {c:24s} {statistics.median(v.values()):16.0f}")
PY
