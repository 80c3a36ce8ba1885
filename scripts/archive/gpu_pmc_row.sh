# SQ instruction-mix counters for one bench_rows.py row (ROW=tso_seg_c5 ...)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_row
cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
S2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
i=0
for set in "$S1" "$S2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_row/p$i -o pmc -- python3 $R/tools/bench_rows.py --rows ${ROW:-tso_seg_c5} --steps 3 --warmup 1 > $R/gpurun_out/pmc_row/p$i.json 2> $R/gpurun_out/pmc_row/p$i.err || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_row/p$i.err; exit 1; }
done
echo done
