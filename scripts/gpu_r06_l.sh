# Round 6, twelfth GPU call: host results by a copy kernel into page-locked
# landing space (NIC_RESULT_LANDING=1) against the runtime's pageable copies;
# the early overlap check now on by default for a batch with nothing else in flight.
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py tests/test_queue_manager.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NIC_RESULT_LANDING=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py > $O/tests_landing.log 2>&1 || { tail -30 $O/tests_landing.log; exit 1; }
tail -2 $O/tests_landing.log
row() {
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for rep in 1 2; do
  for v in 0 1; do
    row hm_pipe_l${v}_$rep NIC_RESULT_LANDING=$v timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
    row pin_pipe_l${v}_$rep NIC_RESULT_LANDING=$v timeout -k 10 180 $S c3 1048576 12 0 device pinned pipelined || exit 1
    row pin_sync_l${v}_$rep NIC_RESULT_LANDING=$v timeout -k 10 180 $S c3 1048576 6 0 device pinned sync || exit 1
  done
  row dev_sync_$rep timeout -k 10 180 $S c3 1048576 20 0 device device sync device || exit 1
  row dev_pipe_$rep timeout -k 10 180 $S c3 1048576 20 0 device device pipelined device || exit 1
done
echo done
