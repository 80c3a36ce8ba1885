set -o pipefail
mkdir -p gpurun_out/prof
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o $TAG -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof/kt_bench.json 2> $R/gpurun_out/prof/kt.err || { tail $R/gpurun_out/prof/kt.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/fetch -o $TAG -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2> $R/gpurun_out/prof/fetch.err || { tail $R/gpurun_out/prof/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/write -o $TAG -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2> $R/gpurun_out/prof/write.err || { tail $R/gpurun_out/prof/write.err; exit 1; }
echo done
