set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/tune_rx.py --rounds 5 --iters 10 --workloads ${WL:-c2,imix,u64} > gpurun_out/tune.json 2> gpurun_out/tune.err; rc=$?
tail -5 gpurun_out/tune.err; exit $rc
