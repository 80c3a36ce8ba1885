# Round 5: deferred RX verify (BatchedQueuePairConfig::defer_rx_verify).
# The GPU tests of the stage first (fuzz against the host resolve and against
# the eager-sum path), then f1 C3 1 M rows with it off (NIC_DEFER_VERIFY=0)
# and on, alternating on one box.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_r05_late.sh'
set -o pipefail
mkdir -p gpurun_out/late
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rx_stage.py tests/test_queue_manager.py -m gpu > gpurun_out/late/tests.log 2>&1 || { tail -30 gpurun_out/late/tests.log; exit 1; }
tail -3 gpurun_out/late/tests.log
B=tools/bin/bench_rx_stage
: > gpurun_out/late/ab.txt
for k in 1 2 3; do
  for v in "eager:NIC_DEFER_VERIFY=0" "late:NIC_DEFER_VERIFY=1"; do
    name=${v%%:*}; envs=${v#*:}
    for mode in pipelined sync; do
      env $envs timeout -k 10 120 $B c3 1048576 12 0 device device $mode device > gpurun_out/late/${name}_${mode}_$k.json 2> gpurun_out/late/${name}_${mode}_$k.err || { tail gpurun_out/late/${name}_${mode}_$k.err; exit 1; }
      echo "$name $mode $(python3 -c "import json;d=json.load(open('gpurun_out/late/${name}_${mode}_$k.json'));print(d['us_median'], d.get('deferred'))")" | tee -a gpurun_out/late/ab.txt
    done
  done
done
echo done
