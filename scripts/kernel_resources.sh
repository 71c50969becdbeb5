# Static resources of every kernel (device-only compile for gfx950): name, group_segment_fixed_size (static LDS;
# must be 0 mod 16 in kernels that also use dynamic LDS), VGPRs, SGPRs.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
for f in "$R"/multiagent_orb_slam2_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off --cuda-device-only --no-gpu-bundle-output -c "$f" -o "$T/$b.co" 2>/dev/null
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/$b.co" | awk '
    /\.group_segment_fixed_size:/ {lds=$2}
    /^ *\.name:/ {name=$2}
    /\.sgpr_count:/ {sgpr=$2}
    /\.vgpr_count:/ {vgpr=$2}
    /\.wavefront_size:/ {printf "%-28s lds %6s vgpr %4s sgpr %4s\n", name, lds, vgpr, sgpr}'
done
rm -rf "$T"
