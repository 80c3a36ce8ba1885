# Round 5: where the fused qm16 drain's time goes (rocprofv3 kernel trace).
set -o pipefail
mkdir -p gpurun_out/qmprof
B=$GRAFT_REPO_ROOT/tools/bin/bench_rx_stage
timeout -k 10 120 $B qm16 1048576 6 0 device device sync device > gpurun_out/qmprof/plain.json 2>&1 || exit 1
cat gpurun_out/qmprof/plain.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt -o qm -- $B qm16 1048576 3 0 device device sync device > $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.err || { tail $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.err; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 200 $B c3 1048576 6 0 device device pipelined device irq > gpurun_out/qmprof/irq.json 2> gpurun_out/qmprof/irq.err || { tail gpurun_out/qmprof/irq.err; exit 1; }
cat gpurun_out/qmprof/irq.json
echo done
