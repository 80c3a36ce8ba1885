#!/bin/bash
# Row f1: the pipelined C3 stage bench and deliver_kernel duration per NICGPU_DLV_RESERVE_CUS value.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f1env
cd /tmp && export TMPDIR=/tmp
for rv in ${RESERVES:-0 8 16 32}; do
  NICGPU_DLV_RESERVE_CUS=$rv timeout -k 10 120 $R/tools/bin/bench_rx_stage c3 1048576 12 0 device device pipelined device > $R/gpurun_out/f1env/r$rv.json 2>&1 || { echo "r$rv bench failed"; exit 1; }
  NICGPU_DLV_RESERVE_CUS=$rv timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f1env/tr_r$rv -o f1 --output-format csv -- $R/tools/bin/bench_rx_stage c3 1048576 6 0 device device pipelined device > $R/gpurun_out/f1env/tr_r$rv.log 2>&1 || { echo "r$rv trace failed"; exit 1; }
  python3 - r$rv <<'PY'
import csv, glob, json, os, sys
v = sys.argv[1]
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/f1env"
j = [l for l in open(f"{R}/{v}.json") if l.startswith("{")][-1]
st = glob.glob(f"{R}/tr_{v}/**/*kernel_stats.csv", recursive=True)[0]
d = [r for r in csv.DictReader(open(st)) if "deliver_kernel" in r["Name"]]
print(v, "pipelined_us", json.loads(j)["us_median"], "deliver_avg_us", [round(float(r["AverageNs"]) / 1e3, 1) for r in d])
PY
done
