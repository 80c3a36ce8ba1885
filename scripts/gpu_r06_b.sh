# Round 6, second GPU call: the bench line at N = 1, the interrupt-replay
# helper A/B (NIC_IRQ_TOUCH) and the HostMemory rows, alternating processes.
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
S=tools/bin/bench_rx_stage
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['roofline']['frac'], d['kernel_us_avg'])"
for k in 0 1 0 1; do
  NIC_IRQ_TOUCH=$k timeout -k 10 180 $S c3 1048576 6 0 device device pipelined device irq > $O/irq_$k.json 2> $O/irq_$k.err || { tail -5 $O/irq_$k.err; exit 1; }
  echo "irq touch=$k: $(tail -1 $O/irq_$k.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['us_median'], d['callback_floor_us'], d.get('phases_us'))")"
done
for m in pipelined sync; do
  timeout -k 10 180 $S c3 1048576 8 0 device hostmem $m > $O/hostmem_$m.json 2> $O/hostmem_$m.err || { tail -5 $O/hostmem_$m.err; exit 1; }
  echo "hostmem $m: $(tail -1 $O/hostmem_$m.json)"
done
echo done
