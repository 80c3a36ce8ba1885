#!/bin/bash
# ICRC timing: production build vs side builds in smart_nic_amd/ab/ (NICGPU_LIB_AB)
set -o pipefail
mkdir -p gpurun_out
for lib in "" smart_nic_amd/ab/*.so; do
  echo "== ${lib:-production}"
  NICGPU_LIB_AB=$lib timeout -k 10 200 python tools/bench_rows.py --rows ${ROWS:-icrc_c2,icrc_c3} --steps 20 2>/dev/null | grep '^{' || exit 1
done
