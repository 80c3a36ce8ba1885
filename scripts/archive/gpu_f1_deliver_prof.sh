# rocprofv3 evidence for the f1 delivery kernel alone (tools/f1_deliver_bench.py,
# C3 1 M, page-aligned 2-KiB RX slots): kernel trace + FETCH_SIZE / WRITE_SIZE
# passes, with the source identity of every GPU source (tools/kernel_sha.py all).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dlvprof
mkdir -p $O
python $R/tools/kernel_sha.py all > $O/kernel_source.sha
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o dlv -- python3 $R/tools/f1_deliver_bench.py --modes= --rounds 2 > $O/attr.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o dlv -- python3 $R/tools/f1_deliver_bench.py --modes= --rounds 1 --iters 3 > /dev/null 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
done
cat $O/attr.json
