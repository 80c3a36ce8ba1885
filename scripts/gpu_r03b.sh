#!/bin/bash
# round 3: the whole GPU suite, then f1 benches (with/without interrupts), then A/B rows vs the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r03b_test.log | tail -5; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r03b_test.log | head; exit $rc; }
for args in "c3 1048576 12 0 device device pipelined device" "c3 1048576 6 0 device device sync device" \
            "c3 1048576 12 0 device pinned pipelined host" "c3 1048576 12 0 device pinned pipelined host irq" \
            "c3 1048576 6 0 device pinned sync host" "c3 1048576 6 0 device pinned sync host irq"; do
  timeout -k 10 120 tools/bin/bench_rx_stage $args 2>/dev/null | grep '^{' | cut -c1-420 || exit 1
done
ROWS=rx_c2,rx_c3,rx_u64 timeout -k 10 600 bash scripts/gpu_ab_rows.sh
