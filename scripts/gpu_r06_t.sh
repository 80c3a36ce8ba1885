# Round 6: SQ counters of the TSO checksum kernel (tools/bench_rows.py rows), one --pmc pass per set.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/bench_rows.py --rows tso_c5 --steps 3 --warmup 1"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p$i -- $B > $O/b$i.json 2> $O/b$i.err || { echo "pmc set $i failed"; tail -5 $O/b$i.err; exit 1; }
  echo "set $i done"
done
echo done
