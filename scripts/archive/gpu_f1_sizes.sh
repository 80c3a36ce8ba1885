# Row f1: batch-size curve of the device-resolved BatchedQueuePair (C3 IMIX,
# pinned descriptor arrays): fixed per-batch cost vs PCIe-bound throughput.
set -o pipefail
mkdir -p gpurun_out
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
: > gpurun_out/rows_f1_sizes.jsonl
for n in 1024 4096 16384 65536 262144 1048576; do
  timeout -k 10 120 ./gpurun_out/bench_rx_stage c3 $n 9 0 device pinned >> gpurun_out/rows_f1_sizes.jsonl 2>> gpurun_out/f1_sizes.err || exit $?
  timeout -k 10 120 ./gpurun_out/bench_rx_stage c3 $n 12 0 device pinned pipelined >> gpurun_out/rows_f1_sizes.jsonl 2>> gpurun_out/f1_sizes.err || exit $?
done
cat gpurun_out/rows_f1_sizes.jsonl
