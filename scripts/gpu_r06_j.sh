# Round 6, tenth GPU call: HostMemory staging by the gather kernel instead of
# the copy engine (NIC_STAGE_GATHER), and the same row with results kept on the
# device (no result downloads sharing the link).
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -k "host_memory or refmem or pipelined" \
  tests/test_rx_stage.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NIC_STAGE_GATHER=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -k "host_memory or refmem or pipelined" \
  tests/test_rx_stage.py > $O/tests_gather.log 2>&1 || { tail -30 $O/tests_gather.log; exit 1; }
tail -2 $O/tests_gather.log
row() {
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d['tx_staged_whole'], d.get('phases_us'))")"
}
for rep in 1 2; do
  for g in 0 1; do
    row hm_pipe_g${g}_$rep NIC_STAGE_GATHER=$g timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
    row hm_pipe_dev_g${g}_$rep NIC_STAGE_GATHER=$g timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined device || exit 1
  done
done
row hm_pipe_g1_b4 NIC_STAGE_GATHER=1 NICGPU_IMG_BLOCKS_PER_CU=4 timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
row hm_sync_g1 NIC_STAGE_GATHER=1 timeout -k 10 180 $S c3 1048576 8 0 device hostmem sync || exit 1
echo done
