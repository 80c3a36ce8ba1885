# Round 6: the segmentation kernel with branch-free edge dwords (buffer stores
# whose out-of-range bytes the hardware drops) — every TSO / segmentation GPU
# test, then the tso_seg_c5 row three times and its SQ instruction counts.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -k "tso or seg" tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 200 python tools/bench_rows.py --rows tso_seg_c5 > $O/tso_$rep.jsonl 2> $O/tso_$rep.err || { tail -5 $O/tso_$rep.err; exit 1; }
  echo "tso_seg_c5: $(python -c "import json; d=json.loads(open('$O/tso_$rep.jsonl').read().strip().splitlines()[-1]); print(d['us_median'], d['roofline_frac'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/bench_rows.py --rows tso_seg_c5 --steps 3 --warmup 1 > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
echo done
