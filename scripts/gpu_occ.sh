# RX kernel at capped occupancy (tuning): U=2 and U=4 variants at 2..4
# blocks per CU, interleaved A/B, then per-wave end stamps of the best ones.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/tune_rx.py --rounds 5 --iters 10 --workloads ${WL:-c2,imix,u64} --variants 0,3,4 \
    --bpcs 0,2,3 --modes auto --no-ceiling > gpurun_out/tune_occ.json 2> gpurun_out/tune_occ.err || { tail -5 gpurun_out/tune_occ.err; exit 1; }
: > gpurun_out/stamps_occ.jsonl
for cfg in "0 0" "3 2" "3 3" "4 2"; do
  set -- $cfg
  timeout -k 10 300 python tools/wave_stamps.py --workloads c2 --variant $1 --bpc $2 >> gpurun_out/stamps_occ.jsonl 2>> gpurun_out/stamps_occ.err || exit 1
done
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/tune_occ.json"))
for w, v in d["workloads"].items():
    print(w, {k: r["us_median"] for k, r in v["results"].items()})
for l in open("gpurun_out/stamps_occ.jsonl"):
    s = json.loads(l); b = s["best"]
    print(s["variant"], "bpc", s["bpc"], "waves", b["waves"], "span", b["span_us"], "end_q", b["end_q"])
PY
