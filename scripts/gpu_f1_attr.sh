# f1 delivery attribution (tools/f1_deliver_bench.py): production, tuning
# modes, gather and the plain copy on the C3 write list; 2-KiB slots and a
# 2112-B slot stride (DRAM channel spread of the destinations).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/f1_deliver_bench.py > gpurun_out/f1attr_2048.json 2> gpurun_out/f1attr.err || { tail gpurun_out/f1attr.err; exit 1; }
cat gpurun_out/f1attr_2048.json
timeout -k 10 200 python tools/f1_deliver_bench.py --slot 2112 --modes 0,1,8 > gpurun_out/f1attr_2112.json 2>> gpurun_out/f1attr.err || { tail gpurun_out/f1attr.err; exit 1; }
cat gpurun_out/f1attr_2112.json
