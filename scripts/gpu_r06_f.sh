# Round 6, sixth GPU call: the PCIe duplex probe (tools/probe_duplex.hip), and
# kernel + copy timelines of the f1 C3 1 M batch on HBM (sync and pipelined)
# and on a HostMemory (pipelined), for where each batch's time goes.
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./tools/bin/probe_duplex > $O/duplex.jsonl 2>&1 || { cat $O/duplex.jsonl; exit 1; }
cat $O/duplex.jsonl
S=tools/bin/bench_rx_stage
for m in sync pipelined; do
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl_hbm_$m -o tl -- \
    $S c3 1048576 10 0 device device $m device > $O/tl_hbm_$m.json 2> $O/tl_hbm_$m.err || { tail -5 $O/tl_hbm_$m.err; exit 1; }
  tail -1 $O/tl_hbm_$m.json
done
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl_hm_pipelined -o tl -- \
  $S c3 1048576 6 0 device hostmem pipelined > $O/tl_hm_pipelined.json 2> $O/tl_hm_pipelined.err || { tail -5 $O/tl_hm_pipelined.err; exit 1; }
tail -1 $O/tl_hm_pipelined.json
find $O -name "*.csv" | head -20
echo done
