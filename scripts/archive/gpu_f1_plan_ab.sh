#!/bin/bash
# f1 asynchronous plan vs the round-2 plan with its wait (NICGPU_F1_SYNC_PLAN=1): alternating
# processes of the pipelined and one-at-a-time C3 1 M stage bench, descriptors and results in HBM.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/f1plan
mkdir -p $O
for i in 1 2 3; do
  for m in 0 1; do
    for mode in pipelined sync; do
      NICGPU_F1_SYNC_PLAN=$m timeout -k 10 120 tools/bin/bench_rx_stage c3 1048576 12 0 device device $mode device > $O/s${m}_${mode}_$i.json 2>&1 || { echo "fail $m $mode"; tail -3 $O/s${m}_${mode}_$i.json; exit 1; }
      python3 -c "import json,sys; j=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('sync_plan', sys.argv[2], sys.argv[3], j['us_median'])" $O/s${m}_${mode}_$i.json $m $mode
    done
  done
done
