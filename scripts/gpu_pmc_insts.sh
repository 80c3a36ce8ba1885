# Instruction-mix PMC for the production RX kernel on C2 (two counter passes).
set -o pipefail
mkdir -p gpurun_out/pmc_i
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_i/p$i -o p$i -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_i/b$i.json 2>$R/gpurun_out/pmc_i/b$i.err || { echo "pmc set $i failed"; tail -5 $R/gpurun_out/pmc_i/b$i.err; exit 1; }
done
find $R/gpurun_out/pmc_i -name "*counter_collection*" | head
