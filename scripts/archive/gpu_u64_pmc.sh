# RX kernel on 4 M x 64 B (bench_rows rx_u64): the LDS and issue counters of
# the small-packet epilogue, one --pmc pass, plus its kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/u64
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o u64 -- python3 $R/tools/bench_rows.py --rows rx_u64 --steps 20 --warmup 3 > $O/row.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/p1 -o u64 -- python3 $R/tools/bench_rows.py --rows rx_u64 --steps 5 --warmup 1 > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d $O/p2 -o u64 -- python3 $R/tools/bench_rows.py --rows rx_u64 --steps 5 --warmup 1 > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 1; }
cat $O/row.json
