# GPU tests (production kernels), then every tuning variant vs the oracle,
# then the variant timing A/B.  Each step has its own time limit; stop at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q --ignore=tests/test_gpu_variants.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_variants.py -x -q > gpurun_out/pytest_variants.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_variants.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python tools/tune_rx.py --rounds 5 --iters 10 --workloads ${WL:-c2,imix,u64} > gpurun_out/tune.json 2> gpurun_out/tune.err
rc=$?; tail -5 gpurun_out/tune.err; exit $rc
