# Round 6, fifth GPU call: do the stage's side streams share hardware queues?
# (7 streams on GPU_MAX_HW_QUEUES=4: a long write-back kernel would hold up the
# check or resolve queued behind it.)  f1 C3 1 M rows at 4 / 8 / 16 queues.
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
S=tools/bin/bench_rx_stage
row() {  # name env... -- args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for q in 4 8 16 4 8; do
  row hm_pipe_q$q GPU_MAX_HW_QUEUES=$q timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
done
for q in 4 8 4 8; do
  row hbm_pipe_q$q GPU_MAX_HW_QUEUES=$q timeout -k 10 180 $S c3 1048576 20 0 device device pipelined device || exit 1
  row hbm_sync_q$q GPU_MAX_HW_QUEUES=$q timeout -k 10 180 $S c3 1048576 20 0 device device sync device || exit 1
done
row hm_sync_q8 GPU_MAX_HW_QUEUES=8 timeout -k 10 180 $S c3 1048576 8 0 device hostmem sync || exit 1
row qm16_q8 GPU_MAX_HW_QUEUES=8 timeout -k 10 180 $S qm16 1048576 8 0 device hostmem sync || exit 1
echo done
