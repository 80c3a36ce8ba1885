# Row f1 (batched QueuePair): the RX-stage GPU tests (fixtures through both
# resolvers, device-vs-host fuzz), then the f1 bench with the device resolve
# and with the host resolve.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_rx_stage.py tests/test_host_cpp.py -m gpu -s > gpurun_out/pytest_f1.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|ok \(|passed|failed" gpurun_out/pytest_f1.log | tail -12; [ $rc -eq 0 ] || exit $rc
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
: > gpurun_out/rows_f1.jsonl
for mode in "device pageable" "device pinned" "device pageable pipelined" "device pinned pipelined" "host pageable"; do
  set -- $mode
  timeout -k 10 300 ./gpurun_out/bench_rx_stage c3 1048576 12 0 $1 $2 ${3:-sync} >> gpurun_out/rows_f1.jsonl 2>> gpurun_out/f1.err || exit $?
  timeout -k 10 300 ./gpurun_out/bench_rx_stage c5 131072 12 0 $1 $2 ${3:-sync} >> gpurun_out/rows_f1.jsonl 2>> gpurun_out/f1.err || exit $?
done
tail -8 gpurun_out/f1.err; cat gpurun_out/rows_f1.jsonl
