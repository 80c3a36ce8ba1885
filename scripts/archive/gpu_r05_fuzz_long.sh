# Round 5: a longer GPU fuzz campaign over the final tree (deferred RX verify
# included): 900 single batches against the host resolve, 150 pipelined
# sequences on HBM and 100 on a HostMemory against eager process_batch, 200
# queue managers against each queue pair alone on the host.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- 'bash scripts/gpu_r05_fuzz_long.sh'
set -o pipefail
mkdir -p gpurun_out/fuzz
g++ -std=c++20 -O2 -Iinclude -Ioracle tests/cpp/rx_stage_gpu_fuzz.cpp -x c oracle/oracle.c -x none -Lsmart_nic_amd -lnic_host -lnicgpu -Wl,-rpath,$PWD/smart_nic_amd -o gpurun_out/fuzz/fuzz 2> gpurun_out/fuzz/build.err || { tail gpurun_out/fuzz/build.err; exit 1; }
F=gpurun_out/fuzz/fuzz
timeout -k 10 300 $F 1001 900 > gpurun_out/fuzz/case.out 2> gpurun_out/fuzz/case.err || { tail gpurun_out/fuzz/case.err; exit 1; }
tail -1 gpurun_out/fuzz/case.out
timeout -k 10 200 $F pipeline 150 > gpurun_out/fuzz/pipe.out 2> gpurun_out/fuzz/pipe.err || { tail gpurun_out/fuzz/pipe.err; exit 1; }
tail -1 gpurun_out/fuzz/pipe.out
timeout -k 10 200 $F pipeline himg 100 > gpurun_out/fuzz/himg.out 2> gpurun_out/fuzz/himg.err || { tail gpurun_out/fuzz/himg.err; exit 1; }
tail -1 gpurun_out/fuzz/himg.out
timeout -k 10 300 $F qm 200 > gpurun_out/fuzz/qm.out 2> gpurun_out/fuzz/qm.err || { tail gpurun_out/fuzz/qm.err; exit 1; }
tail -1 gpurun_out/fuzz/qm.out
echo done
