# Round 5: deferred RX verify in the fused BatchedQueueManager batch — the
# queue-manager GPU tests (fixtures, scale fixture, fused fuzz with deferring
# managers) and the stage's, then qm16 HBM with it off and on, alternating.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash scripts/gpu_r05_late_qm.sh'
set -o pipefail
mkdir -p gpurun_out/lateqm
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_queue_manager.py tests/test_rx_stage.py -m gpu > gpurun_out/lateqm/tests.log 2>&1 || { tail -30 gpurun_out/lateqm/tests.log; exit 1; }
tail -3 gpurun_out/lateqm/tests.log
B=tools/bin/bench_rx_stage
: > gpurun_out/lateqm/ab.txt
for k in 1 2 3; do
  for v in "eager:NIC_DEFER_VERIFY=0" "late:NIC_DEFER_VERIFY=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B qm16 1048576 6 0 device device sync device > gpurun_out/lateqm/${name}_$k.json 2> gpurun_out/lateqm/${name}_$k.err || { tail gpurun_out/lateqm/${name}_$k.err; exit 1; }
    echo "$name qm16 $(python3 -c "import json;d=json.load(open('gpurun_out/lateqm/${name}_$k.json'));print(d['us_median'])")" | tee -a gpurun_out/lateqm/ab.txt
  done
done
echo done
