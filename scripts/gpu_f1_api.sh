# Row f1 pipelined mode: HIP API + kernel + copy trace (no counters), to see
# which host calls stall between the resolve and the DMA writes.
set -o pipefail
mkdir -p gpurun_out/f1api
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d gpurun_out/f1api -o api -- ./gpurun_out/bench_rx_stage c3 1048576 8 0 device ${F1_DESC:-pinned} pipelined > gpurun_out/f1api/bench.log 2>&1 || exit $?
tail -1 gpurun_out/f1api/bench.log
