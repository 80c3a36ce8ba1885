# Round 5: blocks per CU of the batched QueuePair's per-TX kernels (count, fill,
# need, full, relax; NICGPU_QP_BLOCKS_PER_CU, default 8) — the f1 C3 1 M rows
# (HBM descriptors and results, one at a time and pipelined) and qm16, interleaved.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_qpgrid_ab.sh'
set -o pipefail
mkdir -p gpurun_out/qpg
B=tools/bin/bench_rx_stage
for k in 1 2; do
  for g in ${GRIDS:-8 16 4}; do
    for m in sync pipelined; do
      NICGPU_QP_BLOCKS_PER_CU=$g timeout -k 10 120 $B c3 1048576 12 0 device device $m device > gpurun_out/qpg/${g}_${m}_$k.json 2> gpurun_out/qpg/${g}_${m}_$k.err || { tail gpurun_out/qpg/${g}_${m}_$k.err; exit 1; }
      echo "bpc $g $m $(python3 -c "import json;d=json.load(open('gpurun_out/qpg/${g}_${m}_$k.json'));print(d['us_median'])")"
    done
    NICGPU_QP_BLOCKS_PER_CU=$g timeout -k 10 120 $B qm16 1048576 6 0 device device sync device > gpurun_out/qpg/${g}_qm_$k.json 2> gpurun_out/qpg/${g}_qm_$k.err || { tail gpurun_out/qpg/${g}_qm_$k.err; exit 1; }
    echo "bpc $g qm16 $(python3 -c "import json;d=json.load(open('gpurun_out/qpg/${g}_qm_$k.json'));print(d['us_median'])")"
  done
done
echo done
