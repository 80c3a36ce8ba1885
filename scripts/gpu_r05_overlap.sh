# Round 5: the overlapped resolve of submit/collect (a batch's piece sums and
# resolve beside the earlier batches' DMA writes): the pipeline GPU tests, then
# the f1 C3 1 M pipelined rows with and without it (NIC_BENCH_NO_OVERLAP=1).
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_r05_overlap.sh'
set -o pipefail
mkdir -p gpurun_out/ov
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_rx_stage.py -m gpu > gpurun_out/ov/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|overlapped|passed|failed" gpurun_out/ov/tests.log | tail -16; [ $rc -eq 0 ] || exit $rc
B=tools/bin/bench_rx_stage
for k in 1 2; do
  timeout -k 10 120 $B c3 1048576 12 0 device device pipelined device > gpurun_out/ov/on_$k.json 2> gpurun_out/ov/on_$k.err || { tail gpurun_out/ov/on_$k.err; exit 1; }
  cat gpurun_out/ov/on_$k.json
  NIC_BENCH_NO_OVERLAP=1 timeout -k 10 120 $B c3 1048576 12 0 device device pipelined device > gpurun_out/ov/off_$k.json 2> gpurun_out/ov/off_$k.err || { tail gpurun_out/ov/off_$k.err; exit 1; }
  cat gpurun_out/ov/off_$k.json
done
timeout -k 10 120 $B c3 1048576 12 0 device pinned pipelined > gpurun_out/ov/pinned.json 2> gpurun_out/ov/pinned.err || { tail gpurun_out/ov/pinned.err; exit 1; }
cat gpurun_out/ov/pinned.json
echo done
