# Round 6, eleventh GPU call: (1) the single-batch overlap check launched early on
# a normal-priority stream (NIC_CHECK_EARLY) — stage tests with it on, f1 HBM
# rows A/B; (2) HostMemory staging by the gather kernel (NIC_STAGE_GATHER) and
# the HostMemory row with results kept on the device.
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
S=tools/bin/bench_rx_stage
NIC_CHECK_EARLY=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py > $O/tests_early.log 2>&1 || { tail -30 $O/tests_early.log; exit 1; }
tail -2 $O/tests_early.log
NIC_STAGE_GATHER=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -k "host_memory or refmem or pipelined" \
  tests/test_rx_stage.py > $O/tests_gather.log 2>&1 || { tail -30 $O/tests_gather.log; exit 1; }
tail -2 $O/tests_gather.log
row() {
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for rep in 1 2 3; do
  for e in 0 1; do
    row dev_sync_e${e}_$rep NIC_CHECK_EARLY=$e timeout -k 10 180 $S c3 1048576 20 0 device device sync device || exit 1
    row dev_pipe_e${e}_$rep NIC_CHECK_EARLY=$e timeout -k 10 180 $S c3 1048576 20 0 device device pipelined device || exit 1
  done
done
for e in 0 1; do
  row pin_pipe_e${e} NIC_CHECK_EARLY=$e timeout -k 10 180 $S c3 1048576 12 0 device pinned pipelined || exit 1
  row c5_sync_e${e} NIC_CHECK_EARLY=$e timeout -k 10 180 $S c5 131072 6 0 device pinned sync || exit 1
done
for rep in 1 2; do
  for g in 0 1; do
    row hm_pipe_g${g}_$rep NIC_STAGE_GATHER=$g timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
    row hm_pipe_dev_g${g}_$rep NIC_STAGE_GATHER=$g timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined device || exit 1
  done
done
echo done
