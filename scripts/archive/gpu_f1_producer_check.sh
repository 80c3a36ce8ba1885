# Mutation check of the device-descriptor hand-over ordering (rx_stage_gpu_fuzz
# pipeline: a slow device-side producer writes each batch's descriptors on the
# caller's stream just before submit()).  smart_nic_amd/mut/libnic_host.so is
# rx_stage.cpp built without the side stream's wait on ev_submit:
#   sed 's|    if (side) check(nicgpu_stream_wait_event(ps, sl.ev_submit), "nicgpu_stream_wait_event");||' \
#     smart_nic_amd/csrc/host/rx_stage.cpp > smart_nic_amd/csrc/host/rx_stage_mut.cpp
#   (cd smart_nic_amd && g++ -O2 -std=c++20 -fPIC -I../include -shared -o mut/libnic_host.so \
#     csrc/host/{checksum,rss,rx_stage_mut,icrc}.cpp -L. -lnicgpu -Wl,-rpath,'$ORIGIN/..')
# The mutant must fail ("pipelined run differs"); the production library must pass.
set -o pipefail
mkdir -p gpurun_out
g++ -std=c++20 -O2 -Iinclude -Ioracle tests/cpp/rx_stage_gpu_fuzz.cpp -x c oracle/oracle.c -x none -Lsmart_nic_amd -lnic_host -lnicgpu -Wl,-rpath,$PWD/smart_nic_amd -o gpurun_out/fz 2> /dev/null || exit 1
LD_LIBRARY_PATH=$PWD/smart_nic_amd/mut timeout -k 10 200 ./gpurun_out/fz pipeline 40 > gpurun_out/mut.log 2>&1
echo "mutant exit: $?"; tail -3 gpurun_out/mut.log
timeout -k 10 200 ./gpurun_out/fz pipeline 40 > gpurun_out/nomut.log 2>&1
rc=$?; echo "production exit: $rc"; tail -3 gpurun_out/nomut.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rx_stage.py tests/test_gpu_fullsize.py -k "rx_stage or f1_full" -m gpu > gpurun_out/pytest_f1.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_f1.log | tail -2; exit $rc
