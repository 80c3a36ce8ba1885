# Round 6, fourth GPU call: the HostMemory tests after the double mirror, then
# the f1 C3 1 M HostMemory rows A/B — one mirror vs two (NIC_IMAGE_MIRRORS),
# and the image kernels' workgroups per CU (NICGPU_IMG_BLOCKS_PER_CU); the
# segmentation kernel with and without the next frame's loads in flight
# beside the stores (NICGPU_TSO_PREFETCH).
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rx_stage.py tests/test_queue_manager.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "tso or seg" tests > $O/tests_tso.log 2>&1 || { tail -30 $O/tests_tso.log; exit 1; }
tail -3 $O/tests_tso.log
for rep in 1 2; do
  for p in 0 1; do
    NICGPU_TSO_PREFETCH=$p timeout -k 10 200 python tools/bench_rows.py --rows tso_seg_c5 > $O/tso_p${p}_$rep.jsonl 2> $O/tso_p${p}_$rep.err || { tail -5 $O/tso_p${p}_$rep.err; exit 1; }
    echo "tso prefetch=$p: $(python -c "import json; d=json.loads(open('$O/tso_p${p}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['us_median'], d['roofline_frac'])")"
  done
done
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
