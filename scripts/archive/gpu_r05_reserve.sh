# Round 5: the delivery's CU reserve (NICGPU_DLV_RESERVE_CUS: CUs left without
# a delivery block so the next batch's plan and check get wave slots), with the
# RX verifies deferred.  f1 C3 1 M HBM pipelined and one at a time, qm16.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_reserve.sh'
set -o pipefail
mkdir -p gpurun_out/res
B=tools/bin/bench_rx_stage
: > gpurun_out/res/ab.txt
for k in 1 2; do
  for r in 0 8 16 32 48 64; do
    for args in "c3 1048576 12 0 device device pipelined device" "c3 1048576 12 0 device device sync device" "qm16 1048576 6 0 device device sync device"; do
      NICGPU_DLV_RESERVE_CUS=$r timeout -k 10 120 $B $args > gpurun_out/res/one.json 2> gpurun_out/res/one.err || { tail gpurun_out/res/one.err; exit 1; }
      echo "res$r $(echo $args | cut -d' ' -f1,7) $(python3 -c "import json;print(json.load(open('gpurun_out/res/one.json'))['us_median'])")" | tee -a gpurun_out/res/ab.txt
    done
  done
done
echo done
