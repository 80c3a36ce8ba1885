#!/bin/bash
# ICRC waves-per-block A/B: production (16) against side builds with 8 and 12 waves per block
# (smart_nic_amd/ab/icrcN, -DNICGPU_ICRC_WPB=N), alternating processes on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/icrc_wpb
mkdir -p $O
for i in 1 2 3; do
  for v in ${VARIANTS:-16 8 12}; do
    if [ $v = 16 ]; then L=""; else L=$R/smart_nic_amd/ab/icrc$v/libnicgpu.so; fi
    NICGPU_LIB_AB=$L timeout -k 10 120 python3 tools/bench_rows.py --rows icrc_c2,icrc_c3 --steps 20 --warmup 3 > $O/$v.$i.json 2> $O/$v.$i.err || { echo "$v failed"; tail -5 $O/$v.$i.err; exit 1; }
    python3 -c "
import json,sys
for l in open('$O/$v.$i.json'):
    if l.startswith('{'):
        j=json.loads(l)
        for r in j.get('rows',[j]):
            print('$v', r.get('row'), r.get('us_median'), r.get('roofline_frac'))
"
  done
done
