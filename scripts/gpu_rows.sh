# Per-row measurements -> gpurun_out/rows*.jsonl
set -o pipefail
mkdir -p gpurun_out
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
timeout -k 10 300 ./gpurun_out/bench_rx_stage c3 1048576 6 0 device pinned sync > gpurun_out/rows_f1.jsonl || exit $?
timeout -k 10 300 ./gpurun_out/bench_rx_stage c3 1048576 12 0 device pinned pipelined >> gpurun_out/rows_f1.jsonl || exit $?
timeout -k 10 300 ./gpurun_out/bench_rx_stage c5 131072 6 0 device pinned sync >> gpurun_out/rows_f1.jsonl || exit $?
timeout -k 10 300 ./gpurun_out/bench_rx_stage c5 131072 12 0 device pinned pipelined >> gpurun_out/rows_f1.jsonl || exit $?
timeout -k 10 600 python tools/bench_rows.py ${ROWS:+--rows $ROWS} > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; tail -3 gpurun_out/rows.err; cat gpurun_out/rows_f1.jsonl gpurun_out/rows.jsonl; exit $rc
