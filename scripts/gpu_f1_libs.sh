# f1 delivery timing only, over libnicgpu_tune.so and each tuning library in
# AB_LIBS (A/B builds of f1.hip), rounds interleaved inside each process.
set -o pipefail
mkdir -p gpurun_out
for lib in smart_nic_amd/libnicgpu_tune.so ${AB_LIBS}; do
  timeout -k 10 200 python tools/f1_deliver_bench.py --lib $lib ${ATTR_ARGS} >> gpurun_out/f1libs.json 2> gpurun_out/f1libs.err || { tail gpurun_out/f1libs.err; exit 1; }
done
cat gpurun_out/f1libs.json
