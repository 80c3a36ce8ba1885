# f1: GPU tests of the stage, the delivery's cache-policy variants at a
# line-aligned and a misaligned RX base, and the stage's C3 1 M batch with a
# page-aligned and a 16-B-aligned RX ring.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $PT -m gpu tests/test_rx_stage.py tests/test_queue_manager.py tests/test_gpu_fullsize.py ${EXTRA_TESTS} > gpurun_out/f1_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/f1_pytest.log; [ $rc -eq 0 ] || exit $rc
for sh in ${SHIFTS:-0 16}; do
  for lib in smart_nic_amd/libnicgpu_tune.so ${AB_LIBS}; do
    timeout -k 10 200 python tools/f1_deliver_bench.py --lib $lib --modes= --rounds 2 --rx-shift $sh >> gpurun_out/f1libs.json 2>> gpurun_out/f1libs.err || { tail gpurun_out/f1libs.err; exit 1; }
  done
done
for al in 4096 16; do
  for m in pipelined sync; do
    NIC_BENCH_RX_ALIGN=$al timeout -k 10 100 tools/bin/bench_rx_stage c3 1048576 12 0 device device $m device >> gpurun_out/f1stage.json 2>> gpurun_out/f1stage.err || { tail gpurun_out/f1stage.err; exit 1; }
  done
done
cat gpurun_out/f1libs.json gpurun_out/f1stage.json
