#!/bin/bash
# Interrupt replay A/B: the stage bench with TX interrupts on (pinned host descriptors, pipelined and
# one at a time), the production host library against the previous one (smart_nic_amd/ab/oldhost).
set -o pipefail
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then LP=$R/smart_nic_amd/ab/oldhost; else LP=""; fi
    for mode in pipelined sync; do
      LD_LIBRARY_PATH=$LP timeout -k 10 120 tools/bin/bench_rx_stage c3 1048576 6 0 device pinned $mode host irq > /tmp/irq.json 2>&1 || { tail -3 /tmp/irq.json; exit 1; }
      python3 -c "import json; j=[json.loads(l) for l in open('/tmp/irq.json') if l.startswith('{')][-1]; print('$v', '$mode', j['us_median'], j['irq_callbacks'])"
    done
  done
done
