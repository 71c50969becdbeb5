# Round 4, GPU call j: projection / tracking tests, the default bench, a kernel + HIP-API trace of the native per-call
# path (build/host_api_bench: where a single stereo frame's 0.5 ms go), then the bench profile passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4j}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_proj.py tests/test_gpu_tracking.py} -m gpu -x -q -rf --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -c 200 gpurun_out/${T}_bench.log
[ $rb -eq 0 ] || exit $rb
O=gpurun_out/${T}_hapi; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d "$R/$O" -o run -- \
    "$R/build/host_api_bench" "$R/multiagent_orb_slam2_amd/liborbx.so" 60 > $O/hapi.log 2>&1; echo "hapi rc=$?"
[ "${PROF:-1}" = 1 ] && { bash scripts/prof_r4.sh ${T}_prof || exit 1; }
exit $rc
