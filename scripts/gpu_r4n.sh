# Round 4, GPU call n: quadtree stage stamps (make qtprof build), the native per-call path under each image-upload
# mode (ORBX_HOST_H2D 0 banded staging, 1 pageable, 2 one staged copy), then its kernel + HIP-API trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4n}
timeout -k 10 120 python3 scripts/qt_prof.py 128 > gpurun_out/${T}_qtprof.log 2>&1; echo "qtprof rc=$?"; tail -40 gpurun_out/${T}_qtprof.log
for rep in 1 2; do for m in 0 1 2; do
  ORBX_HOST_H2D=$m timeout -k 10 120 "$R/build/host_api_bench" "$R/multiagent_orb_slam2_amd/liborbx.so" 300 \
      > gpurun_out/${T}_hapi_m${m}_${rep}.log 2>&1 || exit $?
  echo "h2d=$m $(tail -1 gpurun_out/${T}_hapi_m${m}_${rep}.log | cut -c1-260)"
done; done
O=gpurun_out/${T}_hapi; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d "$R/$O" -o run -- \
    "$R/build/host_api_bench" "$R/multiagent_orb_slam2_amd/liborbx.so" 60 > $O/hapi.log 2>&1; echo "hapi rc=$?"
