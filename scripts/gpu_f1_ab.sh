#!/bin/bash
# Row f1 A/B: the f1 GPU tests on the production build, then the pipelined C3 stage bench and
# the deliver_kernel's average duration (kernel trace) per deliver-kernel variant
# (smart_nic_amd/ab/<variant>/libnicgpu.so, picked up through LD_LIBRARY_PATH).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f1ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "rx_stage or f1_full or queue_manager" --timeout 300 --timeout-method thread > gpurun_out/f1ab/test.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/f1ab/test.log | tail -3; [ $rc -eq 0 ] || exit $rc
ARGS="c3 1048576 12 0 device device pipelined device"
cd /tmp && export TMPDIR=/tmp
for v in prod ${VARIANTS:-u2 u8 w4 w16u2}; do
  if [ $v = prod ]; then LP=""; else LP=$R/smart_nic_amd/ab/$v; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 120 $R/tools/bin/bench_rx_stage $ARGS > $R/gpurun_out/f1ab/$v.json 2>&1 || { echo "$v bench failed"; tail -3 $R/gpurun_out/f1ab/$v.json; exit 1; }
  LD_LIBRARY_PATH=$LP timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f1ab/tr_$v -o f1 --output-format csv -- $R/tools/bin/bench_rx_stage c3 1048576 6 0 device device pipelined device > $R/gpurun_out/f1ab/tr_$v.log 2>&1 || { echo "$v trace failed"; exit 1; }
  python3 - $v <<'PY'
import csv, glob, json, os, sys
v = sys.argv[1]
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/f1ab"
j = [l for l in open(f"{R}/{v}.json") if l.startswith("{")][-1]
st = glob.glob(f"{R}/tr_{v}/**/*kernel_stats.csv", recursive=True)[0]
d = [r for r in csv.DictReader(open(st)) if "deliver_kernel" in r["Name"]]
print(v, "pipelined_us", json.loads(j)["us_median"], "deliver_avg_us", [round(float(r["AverageNs"]) / 1e3, 1) for r in d])
PY
done
