# Round 2: all -m gpu tests (incl. qp_alias and the long-key / 2^24-table
# batch cases), then the f1 stage rows (host-side cost of the overlap check).
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests -m gpu --ignore=tests/test_gpu_variants.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ROWS=rx_c2 bash scripts/gpu_rows.sh
