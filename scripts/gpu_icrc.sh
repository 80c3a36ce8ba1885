#!/bin/bash
# ICRC (row f4): parity tests, then timing of icrc_c2 / icrc_c3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k icrc --timeout 120 --timeout-method thread > gpurun_out/icrc_test.log 2>&1; rc=$?
tail -8 gpurun_out/icrc_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 20 > gpurun_out/icrc_rows.jsonl 2>&1; rc=$?
grep '^{' gpurun_out/icrc_rows.jsonl; exit $rc
