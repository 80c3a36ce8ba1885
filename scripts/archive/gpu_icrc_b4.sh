#!/bin/bash
# ICRC (row f4) A/B: parity tests on the default kernel, then icrc_c2/icrc_c3 rows and a
# kernel trace per kernel variant (NICGPU_ICRC: b4 = byte tables (default), b4w4, nib).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/icrc_b4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "icrc" --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?
grep -E "passed|failed" $O/test.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/test.log | head; exit $rc; }
for v in ${VARIANTS:-b4 b4w4 nib}; do
  NICGPU_ICRC=$v timeout -k 10 120 python3 tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 20 --warmup 3 > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  echo "== $v"; cat $O/$v.json
done
cd /tmp && export TMPDIR=/tmp
for v in ${PMC_VARIANTS:-b4}; do
  NICGPU_ICRC=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o icrc -- python3 $R/tools/bench_rows.py --rows icrc_c2 --steps 20 --warmup 3 > /dev/null 2> $O/kt_$v.err || { echo "kt $v failed"; tail -5 $O/kt_$v.err; exit 1; }
  for c in FETCH_SIZE SQ_LDS_BANK_CONFLICT; do
    NICGPU_ICRC=$v timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/${c}_$v -o icrc -- python3 $R/tools/bench_rows.py --rows icrc_c2 --steps 5 --warmup 1 > /dev/null 2> $O/${c}_$v.err || { echo "pmc $c $v failed"; tail -5 $O/${c}_$v.err; exit 1; }
  done
done
echo done
