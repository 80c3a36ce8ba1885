# Row f1 with the results left in device memory (results_on_device) and the
# descriptors there too: the RX-stage GPU tests (seeds with bit 1 set and the
# full-size `keep` case take that path), then the f1 bench for every
# combination of host / device descriptors and results, in order and pipelined.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_rx_stage.py tests/test_gpu_fullsize.py -k "rx_stage or f1_full" -m gpu -s \
  > gpurun_out/pytest_keep.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|ok \(|full c|passed|failed" gpurun_out/pytest_keep.log | tail -16; [ $rc -eq 0 ] || exit $rc
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
: > gpurun_out/rows_keep.jsonl
for mode in "pinned sync host" "device sync device" "pinned pipelined host" "device pipelined device" "pinned sync device"; do
  set -- $mode
  timeout -k 10 300 ./gpurun_out/bench_rx_stage c3 1048576 12 0 device $1 $2 $3 >> gpurun_out/rows_keep.jsonl 2>> gpurun_out/keep.err || exit $?
  timeout -k 10 300 ./gpurun_out/bench_rx_stage c5 131072 12 0 device $1 $2 $3 >> gpurun_out/rows_keep.jsonl 2>> gpurun_out/keep.err || exit $?
done
tail -4 gpurun_out/keep.err; cat gpurun_out/rows_keep.jsonl
