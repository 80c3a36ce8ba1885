# Round 6, eighth GPU call: the HostMemory pipelined row under the HIP API
# trace (which host thread waits on what between batches).
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
S=tools/bin/bench_rx_stage
timeout -k 10 240 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o tl -- \
  $S c3 1048576 6 0 device hostmem pipelined > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
tail -1 $O/tl.json
ls -la $O/tl
echo done
