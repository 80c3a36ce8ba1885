#!/bin/bash
# RX hit histogram in a second launch for large batches (NICGPU_RX_SPLIT_HITS=1, production) vs
# inside the RX pass (=0): RX parity + full-size tests with the default, then alternating rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/split
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/test.log | head; exit $rc; }
for i in 1 2; do
  for sp in 1 0; do
    NICGPU_RX_SPLIT_HITS=$sp timeout -k 10 150 python3 tools/bench_rows.py --rows rx_u64,rx_c3,rx_c2 --steps 20 --warmup 3 > $O/r${sp}_$i.json 2> $O/r${sp}_$i.err || { tail -3 $O/r${sp}_$i.err; exit 1; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        r=json.loads(l); print('split', sys.argv[2], r['row'], r['us_region_avg'], r['us_median'], r['roofline_frac'])" $O/r${sp}_$i.json $sp
  done
done
