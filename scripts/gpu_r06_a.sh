# Round 6, first GPU call: the registration probe and heap test, the
# segmentation copy ceiling, the ICRC load-policy A/B (rows + parity), then the
# whole GPU suite.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 60 ./tools/bin/probe_hostreg > $O/probe_hostreg.txt 2>&1; echo "probe rc=$?"
timeout -k 10 60 ./oracle/_ref/rx_stage_test_refmem heap > $O/heap.txt 2>&1 || { echo "heap failed"; cat $O/heap.txt; exit 1; }
tail -2 $O/heap.txt
timeout -k 10 300 python tools/bench_rows.py --rows tso_seg_c5,seg_copy_c5 --steps 10 --warmup 2 > $O/segcopy.jsonl 2> $O/segcopy.err || { tail -5 $O/segcopy.err; exit 1; }
cat $O/segcopy.jsonl
for v in b4 lds b4sc1 ldsmem b4mem b4nt b4 lds b4sc1; do
  NICGPU_ICRC=$v timeout -k 10 200 python tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 10 --warmup 2 > $O/icrc_$v.jsonl 2> $O/icrc_$v.err || { tail -5 $O/icrc_$v.err; exit 1; }
  echo "$v: $(python -c "import json,sys; print([ (d['row'], d['us_median']) for d in map(json.loads, open('$O/icrc_$v.jsonl'))])")"
done
for v in lds b4nt b4sc1; do
  NICGPU_ICRC=$v timeout -k 10 300 python -u -m pytest tests -m gpu -k icrc -x -q --timeout 120 --timeout-method thread > $O/icrc_tests_$v.log 2>&1 || { tail -20 $O/icrc_tests_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/icrc_tests_$v.log)"
done
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; exit $rc
