# f1 delivery stall counters: the production delivery (RSS and not), the
# torch copy of the same bytes and the bare store patterns, one --pmc pass per
# counter group (tools/f1_deliver_bench.py --patterns), kernel stats alongside.
set -o pipefail
mkdir -p gpurun_out/f1stall
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--modes=${MODES:-} --patterns --rounds 1 --iters 2 ${EXTRA_ARGS}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/f1stall/kt -o f1 -- python3 $R/tools/f1_deliver_bench.py $ARGS > $R/gpurun_out/f1stall/kt.json 2> $R/gpurun_out/f1stall/kt.err || { tail -3 $R/gpurun_out/f1stall/kt.err; exit 1; }
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/f1stall/p$i -o f1 -- python3 $R/tools/f1_deliver_bench.py $ARGS > /dev/null 2> $R/gpurun_out/f1stall/p$i.err || { tail -3 $R/gpurun_out/f1stall/p$i.err; exit 1; }
done
echo pmc done
