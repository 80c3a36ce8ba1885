# Round 6: the settled prefix delivered behind the check on the device
# (nicgpu_qp_gate_settled; NIC_DLV_GATE) — the stage tests, then the f1 rows A/B.
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py tests/test_queue_manager.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
row() {
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for rep in 1 2 3; do
  for v in 0 1; do
    row dev_pipe_g${v}_$rep NIC_DLV_GATE=$v timeout -k 10 180 $S c3 1048576 20 0 device device pipelined device || exit 1
  done
done
for v in 0 1; do
  row dev_sync_g${v} NIC_DLV_GATE=$v timeout -k 10 180 $S c3 1048576 20 0 device device sync device || exit 1
  row pin_pipe_g${v} NIC_DLV_GATE=$v timeout -k 10 180 $S c3 1048576 12 0 device pinned pipelined || exit 1
  row hm_pipe_dev_g${v} NIC_DLV_GATE=$v timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined device || exit 1
  row c5_sync_g${v} NIC_DLV_GATE=$v timeout -k 10 180 $S c5 131072 6 0 device pinned sync || exit 1
done
echo done
