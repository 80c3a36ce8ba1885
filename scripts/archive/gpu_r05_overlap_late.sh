# Round 5: the opt-in overlapped resolve (NIC_BENCH_OVERLAP=1) again, now that
# a C3 batch defers its RX verifies (no piece sums beside the delivery), at
# delivery CU reserves 8 (default) and 32.  f1 C3 1 M, HBM, pipelined.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_overlap_late.sh'
set -o pipefail
mkdir -p gpurun_out/ovl
B=tools/bin/bench_rx_stage
: > gpurun_out/ovl/ab.txt
for k in 1 2 3; do
  for v in "off:X=1" "on:NIC_BENCH_OVERLAP=1" "on32:NIC_BENCH_OVERLAP=1 NICGPU_DLV_RESERVE_CUS=32" "off32:NICGPU_DLV_RESERVE_CUS=32"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B c3 1048576 12 0 device device pipelined device > gpurun_out/ovl/${name}_$k.json 2> gpurun_out/ovl/${name}_$k.err || { tail gpurun_out/ovl/${name}_$k.err; exit 1; }
    echo "$name $(python3 -c "import json;d=json.load(open('gpurun_out/ovl/${name}_$k.json'));print(d['us_median'], d['overlapped_resolve'], d['overlap_redone'], d['deferred'])")" | tee -a gpurun_out/ovl/ab.txt
  done
done
echo done
