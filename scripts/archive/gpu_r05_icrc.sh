# Round 5: the pipelined ICRC lane walk (NICGPU_ICRC=pipe: two windows in
# flight per lane) — parity first (every -k icrc test under each variant),
# then alternating-process timing of b4 / pipe / pipe4 / pipemem on C2 and C3.
# Also the fused qm16 kernel trace and the irq row with its wait split.
set -o pipefail
mkdir -p gpurun_out/icrc gpurun_out/qmprof
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for v in pipe pipe4; do
  NICGPU_ICRC=$v timeout -k 10 300 $PT tests -m gpu -k icrc > gpurun_out/icrc/tests_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/icrc/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for v in b4 pipe pipe4 pipemem; do
    NICGPU_ICRC=$v timeout -k 10 120 python tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 10 --warmup 2 > gpurun_out/icrc/rows_${v}_$r.jsonl 2> gpurun_out/icrc/rows_${v}_$r.err || { tail gpurun_out/icrc/rows_${v}_$r.err; exit 1; }
    echo "$v $r $(python -c "import json,sys; print([ (d['row'], d['us_median'], d['roofline_frac']) for d in map(json.loads, open('gpurun_out/icrc/rows_${v}_$r.jsonl'))])")"
  done
done
B=$GRAFT_REPO_ROOT/tools/bin/bench_rx_stage
timeout -k 10 120 $B qm16 1048576 6 0 device device sync device > gpurun_out/qmprof/plain.json 2>&1 || exit 1
cat gpurun_out/qmprof/plain.json
timeout -k 10 200 $B c3 1048576 6 0 device device pipelined device irq > gpurun_out/qmprof/irq.json 2> gpurun_out/qmprof/irq.err || { tail gpurun_out/qmprof/irq.err; exit 1; }
cat gpurun_out/qmprof/irq.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt -o qm -- $B qm16 1048576 3 0 device device sync device > $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.err || { tail $GRAFT_REPO_ROOT/gpurun_out/qmprof/kt.err; exit 1; }
echo done
