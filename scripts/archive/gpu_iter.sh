# Quick kernel iteration: GPU parity tests, variant parity, timing A/B of the
# variants (no ceiling sweep), optional PMC instruction mix (PMC=1).
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 $PT tests -m gpu --ignore=tests/test_gpu_variants.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 $PT tests/test_gpu_variants.py > gpurun_out/pytest_variants.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_variants.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python tools/tune_rx.py --rounds ${ROUNDS:-5} --iters 10 --workloads ${WL:-c2,imix,u64,jumbo} --no-ceiling ${DBG:+--dbg $DBG} ${VARIANTS:+--variants $VARIANTS} ${XPF:+--xpf $XPF} > gpurun_out/tune.json 2> gpurun_out/tune.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tune.err; exit $rc; }
python - <<'EOF'
import json
d = json.load(open("gpurun_out/tune.json"))
for k, v in d["workloads"].items():
    print(k, {n: (r["us_median"], r.get("csum_only_us"), r.get("frac_spec")) for n, r in v["results"].items()})
EOF
if [ -n "$PMC" ]; then
  WLS="${PMC_WLS:-u64 imix}" bash scripts/gpu_pmc_mix.sh || exit 1
  python tools/pmc_mix_summary.py gpurun_out/pmc_mix
fi
echo done
