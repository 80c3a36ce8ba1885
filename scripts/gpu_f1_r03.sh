#!/bin/bash
# row f1 (batched QueuePair stage): GPU tests, then the stage benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "rx_stage or f1" --timeout 300 --timeout-method thread > gpurun_out/f1_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/f1_test.log | tail -15; [ $rc -eq 0 ] || exit $rc
for args in "c3 1048576 6 0 device pinned sync" "c3 1048576 12 0 device device pipelined device" "c3 1048576 6 0 device device sync device" "c5 131072 6 0 device pinned sync"; do
  timeout -k 10 120 tools/bin/bench_rx_stage $args 2>/dev/null | grep '^{' || exit 1
done
