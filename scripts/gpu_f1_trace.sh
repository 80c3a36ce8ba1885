# Kernel trace of the f1 stage's C3 1 M batch (descriptors and results in
# HBM, pipelined): every launch of the steady-state batches with its stream.
set -o pipefail
mkdir -p gpurun_out/f1trace
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/f1trace/kt -o f1 -- $R/tools/bin/bench_rx_stage c3 1048576 8 0 device device ${MODE:-pipelined} device > $R/gpurun_out/f1trace/bench.json 2> $R/gpurun_out/f1trace/bench.err || { tail -3 $R/gpurun_out/f1trace/bench.err; exit 1; }
cat $R/gpurun_out/f1trace/bench.json
