#!/bin/bash
# RX parity (parity + variants + full size), then A/B rows vs the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c_test.log 2>&1; rc=$?
tail -3 gpurun_out/r03c_test.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r03c_test.log | head; exit $rc; }
ROWS=${ROWS:-rx_c2,rx_c3,rx_u64} timeout -k 10 600 bash scripts/gpu_ab_rows.sh || exit 1
# FETCH_SIZE calibration per access shape
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib -o calib -- python3 $R/tools/calib_fetch.py > $R/gpurun_out/calib/order.json 2> $R/gpurun_out/calib/err.log || { tail -5 $R/gpurun_out/calib/err.log; exit 1; }
python3 $R/tools/calib_summary.py $(ls $R/gpurun_out/calib/*counter_collection.csv | head -1) $R/gpurun_out/calib/order.json
