# Round 6, fourth GPU call: the HostMemory tests after the double mirror, then
# the f1 C3 1 M HostMemory rows A/B — one mirror vs two (NIC_IMAGE_MIRRORS),
# and the image kernels' workgroups per CU (NICGPU_IMG_BLOCKS_PER_CU).
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py tests/test_queue_manager.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
row() {  # name env... -- args
  local n=$1; shift
  env "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  echo "$n: $(tail -1 $O/$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['mpkt_s'], d.get('phases_us'))")"
}
for rep in 1 2; do
  for m in 1 2; do
    row pipe_m${m}_b8_$rep NIC_IMAGE_MIRRORS=$m timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
  done
  for b in 2 4; do
    row pipe_m2_b${b}_$rep NICGPU_IMG_BLOCKS_PER_CU=$b timeout -k 10 180 $S c3 1048576 8 0 device hostmem pipelined || exit 1
  done
done
for b in 8 4; do
  row sync_b$b NICGPU_IMG_BLOCKS_PER_CU=$b timeout -k 10 180 $S c3 1048576 8 0 device hostmem sync || exit 1
  row qm16_b$b NICGPU_IMG_BLOCKS_PER_CU=$b timeout -k 10 180 $S qm16 1048576 8 0 device hostmem sync || exit 1
done
echo done
