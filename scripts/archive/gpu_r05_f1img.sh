# Round 5: row f1 on a HostMemory — the rx_stage GPU tests (fixtures on
# FlatHostMemory and on the reference's SimpleHostMemory, the pipelined
# host-memory fuzz, the device-vs-host fuzz with its HostMemory variant) and
# the f1 C3 1 M host-image rows, one batch at a time and pipelined.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_r05_f1img.sh'
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_rx_stage.py -m gpu > gpurun_out/r05_f1img_tests.log 2>&1
rc=$?; tail -16 gpurun_out/r05_f1img_tests.log; [ $rc -eq 0 ] || exit $rc
B=tools/bin/bench_rx_stage
timeout -k 10 200 $B c3 1048576 4 0 device hostmem sync > gpurun_out/r05_f1img_sync.json 2> gpurun_out/r05_f1img_sync.err || { tail gpurun_out/r05_f1img_sync.err; exit 1; }
cat gpurun_out/r05_f1img_sync.json
timeout -k 10 200 $B c3 1048576 8 0 device hostmem pipelined > gpurun_out/r05_f1img_pipe.json 2> gpurun_out/r05_f1img_pipe.err || { tail gpurun_out/r05_f1img_pipe.err; exit 1; }
cat gpurun_out/r05_f1img_pipe.json
echo done
