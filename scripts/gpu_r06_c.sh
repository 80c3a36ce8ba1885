# Round 6: every GPU test, then scripts/gpu_r06_b.sh (bench line, irq A/B, HostMemory rows).
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r06_b.sh
