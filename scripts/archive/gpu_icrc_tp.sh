#!/bin/bash
# ICRC transposed-load variant (NICGPU_ICRC=b4tp): parity with the variant on, then rows per variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/icrc_tp
mkdir -p $O
NICGPU_ICRC=b4tp timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "icrc" --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?
tail -2 $O/test.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/test.log | head; exit $rc; }
for v in ${VARIANTS:-b4 b4tp b4}; do
  NICGPU_ICRC=$v timeout -k 10 120 python3 tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 20 --warmup 3 > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  echo "== $v"; cut -c1-220 $O/$v.json
done
