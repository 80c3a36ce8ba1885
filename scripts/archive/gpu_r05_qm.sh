# Round 5: BatchedQueueManager as one fused device batch — the queue-manager
# GPU tests (fixtures on an HBM image, FlatHostMemory and the reference's
# SimpleHostMemory; the fused-vs-alone fuzz), the rx_stage edges (outgrown
# plan redone once), and the qm16 rows (pinned, device descriptors, host memory).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_r05_qm.sh'
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_memcpy_batch.py tests/test_queue_manager.py "tests/test_rx_stage.py::test_rx_stage_device_limits" -m gpu > gpurun_out/r05_qm_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r05_qm_tests.log; [ $rc -eq 0 ] || exit $rc
B=tools/bin/bench_rx_stage
for kind in pinned device hostmem; do
  timeout -k 10 200 $B qm16 1048576 6 0 device $kind sync device > gpurun_out/r05_qm16_$kind.json 2> gpurun_out/r05_qm16_$kind.err || { tail gpurun_out/r05_qm16_$kind.err; exit 1; }
  cat gpurun_out/r05_qm16_$kind.json
done
# interrupts on, results in HBM: the chunked completion download beside the replay, and the callback floor
timeout -k 10 200 $B c3 1048576 6 0 device device pipelined device irq > gpurun_out/r05_irq.json 2> gpurun_out/r05_irq.err || { tail gpurun_out/r05_irq.err; exit 1; }
cat gpurun_out/r05_irq.json
timeout -k 10 300 $PT tests/test_rx_stage.py -m gpu -k "pipelined or device_resolve" > gpurun_out/r05_irq_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_irq_tests.log; [ $rc -eq 0 ] || exit $rc
echo done
