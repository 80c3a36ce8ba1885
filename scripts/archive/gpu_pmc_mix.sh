# Instruction-mix PMC of the production RX kernel (variant 0) per workload and
# tuple mode (auto = checksum + RSS, none = checksum only): two counter passes
# each, one process per (workload, mode, pass).  -> gpurun_out/pmc_mix/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_mix
cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
S2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
for wl in ${WLS:-u64 imix c2}; do
  for mode in auto none; do
    for p in 1 2; do
      if [ $p = 1 ]; then set="$S1"; else set="$S2"; fi
      o=$R/gpurun_out/pmc_mix/${wl}_${mode}_p$p
      timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $o -o pmc -- python3 $R/tools/tune_rx.py \
        --rounds 1 --iters 3 --workloads $wl --variants ${VARIANT:-0} --modes $mode --no-ceiling > $o.json 2> $o.err \
        || { echo "pmc $wl $mode $p failed"; tail -5 $o.err; exit 1; }
    done
  done
done
echo done
