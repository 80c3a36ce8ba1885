# Row timing of several side libraries against the working tree, interleaved:
# LIBS="e1 e2" -> smart_nic_amd/libnicgpu_e1.so ... (built here beforehand).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/abm.jsonl
for i in $(seq ${ROUNDS:-2}); do
  for side in base $LIBS; do
    if [ $side = base ]; then unset NICGPU_LIB_AB; else export NICGPU_LIB_AB=$PWD/smart_nic_amd/libnicgpu_$side.so; fi
    timeout -k 10 300 python tools/bench_rows.py --rows ${ROWS:-tso_seg_c5} > gpurun_out/abm_one.jsonl 2> gpurun_out/abm.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/abm.err; exit $rc; }
    sed "s/^{/{\"side\": \"$side\", /" gpurun_out/abm_one.jsonl >> gpurun_out/abm.jsonl
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/abm.jsonl"):
    r = json.loads(l); d[(r["row"], r["side"])].append(r["us_median"])
for (row, side), v in sorted(d.items()):
    print(row, side, v)
PY
