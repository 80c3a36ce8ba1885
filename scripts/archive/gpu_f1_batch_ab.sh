# f1 batch A/B: the f1 GPU tests on the tree's library, then the C3 1 M
# HBM-pipelined batch alternating between the tree's libnicgpu.so and the one
# in ab_old/ (built from the previous commit; with libnic_host.so too when
# the host side changed), same box.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $PT -m gpu tests/test_rx_stage.py tests/test_queue_manager.py tests/test_gpu_fullsize.py tests/test_cq_rings.py ${EXTRA_TESTS} > gpurun_out/f1b_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/f1b_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/f1b_ab.jsonl
for rep in 1 2 3; do
  for side in new old; do
    if [ $side = old ]; then export LD_LIBRARY_PATH=$PWD/ab_old; else unset LD_LIBRARY_PATH; fi
    for mode in pipelined sync; do
      timeout -k 10 200 tools/bin/bench_rx_stage c3 1048576 12 0 device device $mode device > gpurun_out/f1b_one.json 2> gpurun_out/f1b.err || { tail gpurun_out/f1b.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/f1b_one.json')); d['side']='$side'; print(json.dumps(d))" >> gpurun_out/f1b_ab.jsonl
    done
  done
done
unset LD_LIBRARY_PATH
python3 - <<'PY'
import json
for l in open('gpurun_out/f1b_ab.jsonl'):
    d=json.loads(l); print(d['side'], d['mode'], d['us_median'])
PY
