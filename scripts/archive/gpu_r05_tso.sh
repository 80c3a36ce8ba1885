# Round 5: TSO segmentation with NICGPU_SEG_PAD (zeros to each segment's next
# 64-B boundary) — the segmentation GPU tests, then the C5 rows with and
# without the flag, twice, interleaved.  Measured slower and removed: this
# recipe ran on that tree (profiles/r05_tso_pad_rejected.jsonl); the flag was not kept.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_tso.sh'
set -o pipefail
mkdir -p gpurun_out/tso
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_parity.py -k "tso" > gpurun_out/tso/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/tso/tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python3 -u tools/bench_rows.py --rows tso_seg_c5,tso_seg_c5_pad --steps 20 --warmup 3 > gpurun_out/tso/rows_$k.jsonl 2> gpurun_out/tso/rows_$k.err || { tail gpurun_out/tso/rows_$k.err; exit 1; }
  cat gpurun_out/tso/rows_$k.jsonl
done
echo done
