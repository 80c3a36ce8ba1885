#!/bin/bash
# same-box A/B: production build vs smart_nic_amd/ab/*.so on bench_rows rows, 3 alternating rounds
set -o pipefail
mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "" smart_nic_amd/ab/*.so; do
    echo "== round $round ${lib:-production}"
    NICGPU_LIB_AB=$lib timeout -k 10 200 python tools/bench_rows.py --rows ${ROWS:-rx_c2,rx_c3,rx_u64} --steps 20 2>/dev/null | grep '^{' | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['row'], r['us_median'], r.get('us_region_avg'), r.get('roofline_frac'))" || exit 1
  done
done
