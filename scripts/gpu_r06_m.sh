# Round 6: the RX variants on 64-B and IMIX batches (deeper per-wave batches,
# U=4, at several blocks-per-CU caps) against production — VERDICT item 7.
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 500 python tools/tune_rx.py --rounds 5 --iters 10 --workloads u64,imix --variants 0,1,2,6,7 \
  --modes auto --bpcs 0,2,3 --no-ceiling > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/r06m/tune.json'))
for w,wl in d['workloads'].items():
    for k,v in wl['results'].items():
        print(w, k, v if not isinstance(v, dict) else {kk: v[kk] for kk in list(v)[:6]})
PY
echo done
