mkdir -p gpurun_out
timeout -k 10 200 python tools/wave_stamps.py --workloads c2 > gpurun_out/stamps_c2.jsonl 2> gpurun_out/stamps.err && \
timeout -k 10 200 python tools/wave_stamps.py --workloads c2 --dbg 8192 >> gpurun_out/stamps_c2.jsonl 2>> gpurun_out/stamps.err && \
timeout -k 10 200 python tools/wave_stamps.py --workloads c2 >> gpurun_out/stamps_c2.jsonl 2>> gpurun_out/stamps.err
