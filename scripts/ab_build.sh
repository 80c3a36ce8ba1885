# Build the side library for a same-box A/B: smart_nic_amd/libnicgpu_ab.so from
# git revision ${REV:-HEAD} (run here, on the CPU, before scripts/gpu_ab.sh).
set -e
REV=${REV:-HEAD}
tmp=$(mktemp -d)
git show "$REV:smart_nic_amd/csrc/nicgpu.hip" > "$tmp/nicgpu.hip"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Iinclude -Ismart_nic_amd/csrc -shared \
  -o smart_nic_amd/libnicgpu_ab.so "$tmp/nicgpu.hip"
rm -rf "$tmp"
echo "built smart_nic_amd/libnicgpu_ab.so from $REV"
