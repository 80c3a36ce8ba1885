# Round 5: overlapped resolve A/B — without / with it (NIC_BENCH_OVERLAP=1),
# and CUs kept free of delivery blocks (NICGPU_DLV_RESERVE_CUS) so the next
# batch's plan, sums and resolve find wave slots beside the delivery.
# f1 C3 1 M, HBM descriptors and results, pipelined.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_overlap_ab.sh'
set -o pipefail
mkdir -p gpurun_out/ov2
B=tools/bin/bench_rx_stage
for k in 1 2; do
  for v in "off8:X=1" "on8:NIC_BENCH_OVERLAP=1" "on32:NIC_BENCH_OVERLAP=1 NICGPU_DLV_RESERVE_CUS=32" "on64:NIC_BENCH_OVERLAP=1 NICGPU_DLV_RESERVE_CUS=64" "on96:NIC_BENCH_OVERLAP=1 NICGPU_DLV_RESERVE_CUS=96" "off48:NICGPU_DLV_RESERVE_CUS=48"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B c3 1048576 12 0 device device pipelined device > gpurun_out/ov2/${name}_$k.json 2> gpurun_out/ov2/${name}_$k.err || { tail gpurun_out/ov2/${name}_$k.err; exit 1; }
    echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/ov2/${name}_$k.json'));print(d['us_median'], d['phases_us']['check'])")"
  done
done
echo done
