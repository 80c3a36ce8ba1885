# Round 5: where the f1 C3 1 M pipelined batch's time goes (HBM descriptors and
# results): the row, then a rocprofv3 kernel trace of the same command.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_f1prof.sh'
set -o pipefail
mkdir -p gpurun_out/f1prof
B=$GRAFT_REPO_ROOT/tools/bin/bench_rx_stage
timeout -k 10 120 $B c3 1048576 12 0 device device pipelined device > gpurun_out/f1prof/plain.json 2> gpurun_out/f1prof/plain.err || { tail gpurun_out/f1prof/plain.err; exit 1; }
cat gpurun_out/f1prof/plain.json
cd /tmp && export TMPDIR=/tmp
NICGPU_DLV_RESERVE_CUS=${RES:-8} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/f1prof/kt -o f1 -- $B c3 1048576 12 0 device device pipelined device > $GRAFT_REPO_ROOT/gpurun_out/f1prof/kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/f1prof/kt.err || { tail $GRAFT_REPO_ROOT/gpurun_out/f1prof/kt.err; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/f1prof/kt.json
echo done
