# One GPU call: production tests, variant parity, smoke, bench line, rocprofv3
# kernel-trace stats and the two PMC traffic passes.  Every GPU step has its own
# time limit; the script stops at the first failure.
#   TAG=r01b /usr/local/graft/bin/gpurun --timeout 1100 -- 'bash scripts/gpu_round.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
mkdir -p gpurun_out/prof
python tools/kernel_sha.py rx > gpurun_out/prof/kernel_source.sha
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT tests -m gpu --ignore=tests/test_gpu_variants.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $PT tests/test_gpu_variants.py > gpurun_out/pytest_variants.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_variants.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o $TAG -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof/kt_bench.json 2> $R/gpurun_out/prof/kt.err || { tail $R/gpurun_out/prof/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/fetch -o $TAG -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2> $R/gpurun_out/prof/fetch.err || { tail $R/gpurun_out/prof/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/write -o $TAG -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2> $R/gpurun_out/prof/write.err || { tail $R/gpurun_out/prof/write.err; exit 1; }
cd $R
if [ -n "$TUNE" ]; then
  timeout -k 10 500 python tools/tune_rx.py --rounds 5 --iters 10 --workloads ${WL:-c2,imix,u64,jumbo} > gpurun_out/tune.json 2> gpurun_out/tune.err
  rc=$?; tail -5 gpurun_out/tune.err; [ $rc -eq 0 ] || exit $rc
fi
echo done
