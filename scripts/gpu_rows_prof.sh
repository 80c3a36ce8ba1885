# rocprofv3 evidence for every §8 row: per row of tools/bench_rows.py a
# kernel-trace --stats run and two PMC passes (FETCH_SIZE, WRITE_SIZE; separate
# runs, no tracing beside --pmc), plus a kernel trace of the f1 stage
# (tools/bench_rx_stage, C3 1 M, device descriptors and results, pipelined).
# Summarise with: python tools/rows_prof_summary.py gpurun_out/rows_prof TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r02r}
O=$R/gpurun_out/rows_prof
mkdir -p $O
python $R/tools/kernel_sha.py all > $O/kernel_source.sha
g++ -std=c++20 -O2 -I$R/include $R/tools/bench_rx_stage.cpp -L$R/smart_nic_amd -lnic_host -lnicgpu \
    -Wl,-rpath,"$R/smart_nic_amd" -o $O/bench_rx_stage || exit 1
cd /tmp && export TMPDIR=/tmp
for row in ${ROWS:-rx_c2 rx_c3 rx_u64 rx_l34_c2 rss_c2 rss_c3 icrc_c2 icrc_c3 tso_c5 tso_seg_c5}; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$row -o $TAG -- python3 $R/tools/bench_rows.py --rows $row --steps 20 --warmup 3 > $O/$row.json 2> $O/kt_$row.err || { echo "kt $row failed"; tail -5 $O/kt_$row.err; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/${c}_$row -o $TAG -- python3 $R/tools/bench_rows.py --rows $row --steps 5 --warmup 1 > /dev/null 2> $O/${c}_$row.err || { echo "pmc $c $row failed"; tail -5 $O/${c}_$row.err; exit 1; }
  done
  echo "row $row done"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_f1 -o $TAG -- $O/bench_rx_stage c3 1048576 12 0 device device pipelined device > $O/f1.json 2> $O/kt_f1.err || { echo "kt f1 failed"; tail -5 $O/kt_f1.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/${c}_f1 -o $TAG -- $O/bench_rx_stage c3 1048576 4 0 device device pipelined device > /dev/null 2> $O/${c}_f1.err || { echo "pmc $c f1 failed"; tail -5 $O/${c}_f1.err; exit 1; }
done
cat $O/f1.json
echo done
