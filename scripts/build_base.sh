# Build the HEAD sources' library into build/base/liborbx.so (the A/B baseline of an uncommitted change)
set -e
T=$(mktemp -d); trap 'rm -rf $T' EXIT
git archive HEAD multiagent_orb_slam2_amd/csrc include | tar -x -C $T
for f in $T/multiagent_orb_slam2_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-fast-math -I$T/include -c $f -o ${f%.hip}.o &
done
wait
mkdir -p build/base
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/base/liborbx.so $T/multiagent_orb_slam2_amd/csrc/*.o -ldl 2>&1 | grep -v hip-link || true
ls -la build/base/liborbx.so
