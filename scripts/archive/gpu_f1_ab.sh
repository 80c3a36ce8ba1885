# f1 delivery A/B: the f1 GPU tests on the production build, then the
# delivery attribution on libnicgpu_tune.so and on each extra tuning library
# named in AB_LIBS (built in-tree beforehand), then the stage's C3 1 M batch.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 120 $PT -m gpu tests/test_gpu_unaligned.py > gpurun_out/f1_unaligned.log 2>&1 || { tail -20 gpurun_out/f1_unaligned.log; exit 1; }
timeout -k 10 500 $PT -m gpu tests/test_rx_stage.py tests/test_queue_manager.py tests/test_gpu_fullsize.py ${EXTRA_TESTS} > gpurun_out/f1_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/f1_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in smart_nic_amd/libnicgpu_tune.so ${AB_LIBS}; do
  timeout -k 10 300 python tools/f1_deliver_bench.py --lib $lib ${ATTR_ARGS} >> gpurun_out/f1attr.json 2> gpurun_out/f1attr.err || { tail gpurun_out/f1attr.err; exit 1; }
done
cat gpurun_out/f1attr.json
for mode in pipelined sync; do
  timeout -k 10 200 tools/bin/bench_rx_stage c3 1048576 12 0 device device $mode device > gpurun_out/f1_c3_$mode.json 2> gpurun_out/f1_c3.err || { tail gpurun_out/f1_c3.err; exit 1; }
  cat gpurun_out/f1_c3_$mode.json
done
