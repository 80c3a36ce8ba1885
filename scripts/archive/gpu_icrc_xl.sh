# ICRC A/B: every ICRC GPU test with the coalesced-load kernel (NICGPU_ICRC=xl),
# then the C2 / C3 rows for the lane walk (b4), xl, and their loads alone.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
# the variants live in commit 9e1bbfe (reverted from production); check it out to rerun
for tv in ${TESTVARS:-xl}; do
  NICGPU_ICRC=$tv timeout -k 10 300 $PT -m gpu -k icrc tests/ > gpurun_out/icrc_${tv}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/icrc_${tv}_pytest.log; [ $rc -eq 0 ] || exit $rc
done
for v in ${VARS:-b4 xl xlmem b4mem xl b4}; do
  NICGPU_ICRC=$v timeout -k 10 200 python tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 10 > gpurun_out/icrc_$v.json 2> gpurun_out/icrc_$v.err || { tail gpurun_out/icrc_$v.err; exit 1; }
  echo "== $v"; cat gpurun_out/icrc_$v.json
done
