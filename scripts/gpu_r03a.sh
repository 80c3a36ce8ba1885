#!/bin/bash
# round 3: ICRC nibble kernel + device-path limits, then ICRC timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "icrc or rx_stage" --timeout 200 --timeout-method thread > gpurun_out/r03a_test.log 2>&1; rc=$?
tail -15 gpurun_out/r03a_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 20 > gpurun_out/r03a_rows.jsonl 2>&1; rc=$?
cat gpurun_out/r03a_rows.jsonl | tail -5; exit $rc
