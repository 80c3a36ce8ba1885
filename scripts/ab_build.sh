# Build the side library for a same-box A/B: smart_nic_amd/libnicgpu_ab.so from
# git revision ${REV:-HEAD} (run here, on the CPU, before scripts/gpu_ab.sh).
# Revisions before the round-4 split have one source, csrc/nicgpu.hip.
set -e
REV=${REV:-HEAD}
tmp=$(mktemp -d)
git archive "$REV" smart_nic_amd/csrc include | tar -x -C "$tmp"
if [ -f "$tmp/smart_nic_amd/csrc/nicgpu.hip" ]; then
  srcs="$tmp/smart_nic_amd/csrc/nicgpu.hip"
else
  srcs=$(for u in runtime rss rx tso icrc f1; do echo "$tmp/smart_nic_amd/csrc/$u.hip"; done)
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -I"$tmp/include" -I"$tmp/smart_nic_amd/csrc" -shared \
  -o smart_nic_amd/libnicgpu_ab.so $srcs
rm -rf "$tmp"
echo "built smart_nic_amd/libnicgpu_ab.so from $REV"
