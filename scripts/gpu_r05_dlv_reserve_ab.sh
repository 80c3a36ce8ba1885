# Round 5: CUs kept free of delivery blocks (NICGPU_DLV_RESERVE_CUS, default 8)
# for the next batch's plan kernels, on the f1 C3 1 M pipelined row (HBM
# descriptors and results) after the per-TX kernels went to 4 blocks per CU.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_dlv_reserve_ab.sh'
set -o pipefail
mkdir -p gpurun_out/dres
B=tools/bin/bench_rx_stage
for k in 1 2; do
  for r in 8 0 24 48; do
    for m in pipelined sync; do
      NICGPU_DLV_RESERVE_CUS=$r timeout -k 10 120 $B c3 1048576 12 0 device device $m device > gpurun_out/dres/${r}_${m}_$k.json 2> gpurun_out/dres/${r}_${m}_$k.err || { tail gpurun_out/dres/${r}_${m}_$k.err; exit 1; }
      echo "reserve $r $m $(python3 -c "import json;d=json.load(open('gpurun_out/dres/${r}_${m}_$k.json'));print(d['us_median'])")"
    done
  done
done
echo done
