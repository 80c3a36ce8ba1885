# Round 5 same-box A/B: the tree's libraries against ab_old/ (a previous
# commit's libnicgpu.so + libnic_host.so), alternating, on the f1 C3 1 M rows
# (HBM descriptors and results, pipelined and one at a time) and qm16 (HBM
# descriptors).  No tests (run them on the tree first).
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash scripts/gpu_r05_ab.sh'
set -o pipefail
# (ab_old/ must travel: a missing directory would silently load the tree's libraries through the rpath)
[ -f ab_old/libnicgpu.so ] && [ -f ab_old/libnic_host.so ] || { echo "ab_old/ missing on the box"; exit 1; }
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.txt
for rep in 1 2 3; do
  for side in new old; do
    if [ $side = old ]; then export LD_LIBRARY_PATH=$PWD/ab_old; else unset LD_LIBRARY_PATH; fi
    for args in "c3 1048576 12 0 device device pipelined device" "c3 1048576 12 0 device device sync device" "qm16 1048576 6 0 device device sync device"; do
      timeout -k 10 120 tools/bin/bench_rx_stage $args > gpurun_out/ab/one.json 2> gpurun_out/ab/one.err || { tail gpurun_out/ab/one.err; exit 1; }
      echo "$side $(echo $args | cut -d' ' -f1,7) $(python3 -c "import json;print(json.load(open('gpurun_out/ab/one.json'))['us_median'])")" | tee -a gpurun_out/ab/ab.txt
    done
  done
done
unset LD_LIBRARY_PATH
echo done
