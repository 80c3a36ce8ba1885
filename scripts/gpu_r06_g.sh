# Round 6, seventh GPU call: host-image staging on its own stream (NIC_STAGE_STREAM)
# — the HostMemory tests, the f1 C3 1 M HostMemory pipelined row A/B, and a
# kernel + copy timeline of the new default.
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
S=tools/bin/bench_rx_stage
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py tests/test_queue_manager.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() {
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for rep in 1 2; do
  for v in 0 1; do
    row hm_pipe_stage${v}_$rep NIC_STAGE_STREAM=$v timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
  done
done
row qm16_hm NIC_STAGE_STREAM=1 timeout -k 10 180 $S qm16 1048576 4 0 device hostmem sync device || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl_hm_pipelined -o tl -- \
  $S c3 1048576 6 0 device hostmem pipelined > $O/tl_hm_pipelined.json 2> $O/tl_hm_pipelined.err || { tail -5 $O/tl_hm_pipelined.err; exit 1; }
tail -1 $O/tl_hm_pipelined.json
echo done
