#!/bin/bash
# RX tiles dealt by per-group counters (NICGPU_RX_DYN=1, variants 3/4) against the fixed round
# robin: every tuning variant bit-exact (incl. the DYN ones), RX parity with DYN on, then
# alternating C2 bench processes (same box) and RX rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dyn
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_variants.py > $O/variants.log 2>&1; rc=$?
tail -2 $O/variants.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/variants.log | head; exit $rc; }
NICGPU_RX_DYN=1 timeout -k 10 400 $PT tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > $O/parity.log 2>&1; rc=$?
tail -2 $O/parity.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/parity.log | head; exit $rc; }
for i in 1 2 3; do
  for d in 0 1; do
    NICGPU_RX_DYN=$d timeout -k 10 150 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-rows > $O/b${d}_$i.json 2> $O/b${d}_$i.err || { tail -3 $O/b${d}_$i.err; exit 1; }
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('dyn', sys.argv[2], 'us_avg', j['kernel_us_avg'], 'us_med', j['kernel_us_median'], 'frac', j['roofline']['frac'], 'ceil', j['roofline']['frac_of_ceiling'], j['checks'])" $O/b${d}_$i.json $d
  done
done
for d in 0 1; do
  NICGPU_RX_DYN=$d timeout -k 10 150 python3 tools/bench_rows.py --rows rx_c2,rx_l34_c2 --steps 20 --warmup 3 > $O/rows$d.json 2> $O/rows$d.err || { tail -3 $O/rows$d.err; exit 1; }
  echo "rows dyn=$d"; cat $O/rows$d.json
done
echo done
