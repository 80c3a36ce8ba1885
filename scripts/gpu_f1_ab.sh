# Same-box A/B of the f1 stage: smart_nic_amd/ab/{libnicgpu,libnic_host}.so (A,
# built from HEAD in a git worktree) against the working tree's libraries (B),
# alternating processes (LD_LIBRARY_PATH beats the driver's RUNPATH); the RX-stage GPU tests first.
set -o pipefail
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_rx_stage.py tests/test_gpu_fullsize.py -k "rx_stage or f1_full" -m gpu \
  > gpurun_out/pytest_f1.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_f1.log | tail -3; [ $rc -eq 0 ] || exit $rc
g++ -std=c++20 -O2 -Iinclude tools/bench_rx_stage.cpp -Lsmart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$PWD/smart_nic_amd" -o gpurun_out/bench_rx_stage || exit 1
: > gpurun_out/f1_ab.jsonl
for i in 1 2 3; do
  for side in A B; do
    if [ $side = A ]; then export LD_LIBRARY_PATH=$PWD/smart_nic_amd/ab; else unset LD_LIBRARY_PATH; fi
    if [ "${MODESET:-}" = pinned1m ]; then set -- "1048576 12 0 device pinned pipelined" "1048576 9 0 device pinned sync"
    else set -- "1024 12 0 device pinned pipelined" "65536 9 0 device pinned sync" "1048576 12 0 device device pipelined device" "1048576 9 0 device device sync device"; fi
    for mode in "$@"; do
      timeout -k 10 120 ./gpurun_out/bench_rx_stage c3 $mode 2>> gpurun_out/f1_ab.err | sed "s/^{/{\"side\": \"$side\", /" >> gpurun_out/f1_ab.jsonl || exit 1
    done
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/f1_ab.jsonl"):
    r = json.loads(l)
    d[(r["tx_descriptors"], r["descriptors"], r["mode"], r["side"])].append(r["us_median"])
for k, v in sorted(d.items()):
    print(k, v)
PY
