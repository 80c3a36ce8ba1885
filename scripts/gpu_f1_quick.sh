#!/bin/bash
# row f1: GPU tests (fuzz incl. interrupt replay, pipeline, full size, limits), then the stage
# bench with and without interrupt callbacks, then the kernel trace + PMC of the pipelined batch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "rx_stage or f1_full" --timeout 300 --timeout-method thread > gpurun_out/f1q_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/f1q_test.log | tail -12; [ $rc -eq 0 ] || exit $rc
for args in "c3 1048576 12 0 device device pipelined device" "c3 1048576 6 0 device device sync device" \
            "c3 1048576 12 0 device pinned pipelined host" "c3 1048576 12 0 device pinned pipelined host irq" \
            "c3 1048576 6 0 device pinned sync host" "c3 1048576 6 0 device pinned sync host irq"; do
  timeout -k 10 120 tools/bin/bench_rx_stage $args 2>/dev/null | grep '^{' || exit 1
done
bash scripts/gpu_f1_prof_r03.sh 2>&1 | tail -20
