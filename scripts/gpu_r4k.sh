# Round 4, GPU call k: extraction / projection / tracking / ordering tests, the bench with the blur fused into the
# resize launches and without (A/B in one call), a kernel + HIP-API trace of the native per-call path, the profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4k}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_extract.py tests/test_gpu_proj.py tests/test_gpu_tracking.py tests/test_gpu_ordering.py} \
    -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for f in 1 0 1; do
  ORBX_BLUR_FUSED=$f timeout -k 10 400 python -u bench.py --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd \
      --host-fed-steps 0 > gpurun_out/${T}_bench_f$f.log 2>&1 || exit $?
  echo "fused=$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_f$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench_f$f.log)"
done
O=gpurun_out/${T}_hapi; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d "$R/$O" -o run -- \
    "$R/build/host_api_bench" "$R/multiagent_orb_slam2_amd/liborbx.so" 60 > $O/hapi.log 2>&1; echo "hapi rc=$?"
[ "${PROF:-1}" = 1 ] && { bash scripts/prof_r4.sh ${T}_prof || exit 1; }
exit $rc
