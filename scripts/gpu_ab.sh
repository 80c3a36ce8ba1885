# Same-box A/B of kernel rows: the working-tree libnicgpu.so (B) against
# libnicgpu_ab.so (A, scripts/ab_build.sh), alternating A B A B ... processes.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for i in $(seq ${ROUNDS:-3}); do
  for side in A B; do
    if [ $side = A ]; then export NICGPU_LIB_AB=$PWD/smart_nic_amd/libnicgpu_ab.so; else unset NICGPU_LIB_AB; fi
    timeout -k 10 300 python tools/bench_rows.py --rows ${ROWS:-icrc_c2} > gpurun_out/ab_$side.jsonl 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab.err; exit $rc; }
    sed "s/^{/{\"side\": \"$side\", /" gpurun_out/ab_$side.jsonl >> gpurun_out/ab.jsonl
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab.jsonl"):
    r = json.loads(l); d[(r["row"], r["side"])].append(r["us_median"])
for (row, side), v in sorted(d.items()):
    print(row, side, "median us per process:", v)
PY
