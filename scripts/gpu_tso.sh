# GPU parity tests, then the per-row kernel measurements (ROWS=... to select)
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests -m gpu --ignore=tests/test_gpu_variants.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 600 python tools/bench_rows.py --rows ${ROWS:-tso_c5,tso_seg_c5} > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
rc=$?; tail -3 gpurun_out/rows.err; cat gpurun_out/rows.jsonl; exit $rc
