# TSO segmentation A/B: the segmentation GPU tests on the tree's library, then
# the tso_seg_c5 row alternating with ab_old/libnicgpu.so (NICGPU_LIB_AB), same box.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT -m gpu -k "tso or seg" tests/ > gpurun_out/tso_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/tso_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/tso_ab.jsonl
for rep in 1 2 3; do
  for side in new old; do
    if [ $side = old ]; then export NICGPU_LIB_AB=$PWD/ab_old/libnicgpu.so; else unset NICGPU_LIB_AB; fi
    timeout -k 10 200 python tools/bench_rows.py --rows ${ROWS:-tso_seg_c5} --steps 20 > gpurun_out/tso_one.json 2> gpurun_out/tso.err || { tail gpurun_out/tso.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/tso_one.json'):
    d=json.loads(l); d['side']='$side'; print(json.dumps(d))" >> gpurun_out/tso_ab.jsonl
  done
done
unset NICGPU_LIB_AB
python3 -c "
import json
for l in open('gpurun_out/tso_ab.jsonl'):
    d=json.loads(l); print(d['side'], d['row'], d['us_region_avg'], d['us_median'])"
