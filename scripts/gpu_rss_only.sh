# Header-only RSS kernel: the RX parity tests (every gpu_rx call also runs the
# batch without checksums and compares), the IMIX RSS-only test, the f1 tests
# (whose dispatch uses it), then the rss rows beside rx rows and the f1 rows.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_rx_stage.py -m gpu > gpurun_out/pytest_rss.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/pytest_rss.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_rows.py --rows rss_c2,rss_c3,rx_c2,rx_c3 > gpurun_out/rows_rss.jsonl 2> gpurun_out/rows_rss.err || exit $?
cat gpurun_out/rows_rss.jsonl
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
: > gpurun_out/rows_f1_rss.jsonl
for mode in "pinned sync host" "device sync device" "device pipelined device"; do
  set -- $mode
  timeout -k 10 300 ./gpurun_out/bench_rx_stage c3 1048576 12 0 device $1 $2 $3 >> gpurun_out/rows_f1_rss.jsonl 2>> gpurun_out/f1_rss.err || exit $?
done
cat gpurun_out/rows_f1_rss.jsonl
