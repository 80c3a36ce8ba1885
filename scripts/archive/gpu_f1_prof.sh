# Row f1: kernel-level profile of the device-resolved batched QueuePair on
# C3 (1 M IMIX descriptors) — which kernels and copies make up a batch.
set -o pipefail
mkdir -p gpurun_out/f1prof
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/f1prof -o f1 -- ./gpurun_out/bench_rx_stage c3 ${F1_N:-1048576} 3 0 device ${F1_DESC:-pageable} ${F1_MODE:-sync} > gpurun_out/f1prof/bench.log 2>&1 || exit $?
find gpurun_out/f1prof -name "*stats.csv" | head; cat gpurun_out/f1prof/bench.log | tail -3
