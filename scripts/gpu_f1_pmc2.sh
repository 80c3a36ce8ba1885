# f1 delivery: machinery-only modes and SQ instruction counters of the production delivery
set -o pipefail
mkdir -p gpurun_out/f1pmc
timeout -k 10 200 python tools/f1_deliver_bench.py --modes 0,7,39,32 --rounds 2 > gpurun_out/f1attr_mach.json 2> gpurun_out/f1attr.err || { tail gpurun_out/f1attr.err; exit 1; }
cat gpurun_out/f1attr_mach.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/f1pmc/p$i -o f1 -- python3 $R/tools/f1_deliver_bench.py --modes 0,32 --rounds 1 --iters 2 > /dev/null 2> $R/gpurun_out/f1pmc/p$i.err || { tail -3 $R/gpurun_out/f1pmc/p$i.err; exit 1; }
done
echo pmc done
