# Round 4, first GPU call: the hipFree experiment, the host-API latency bisect (r2z .. r3s builds and this tree, one
# native driver), the GPU suite, the default bench.  Each GPU step has its own time limit; a fault, abort or time limit
# ends the script (pytest failures (rc 1) do not: the bench still runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4a}
timeout -k 10 60 ./build/free_sync > gpurun_out/${T}_free_sync.log 2>&1 || exit $?
cat gpurun_out/${T}_free_sync.log
for c in dff1580 6d59bcc 7b6d68d 1a5e409; do
  timeout -k 10 120 ./build/host_api_bench build/bisect/$c/liborbx.so 300 > gpurun_out/${T}_hostapi_$c.log 2>&1 || exit $?
done
timeout -k 10 120 ./build/host_api_bench multiagent_orb_slam2_amd/liborbx.so 300 > gpurun_out/${T}_hostapi_head.log 2>&1 || exit $?
grep -h frames_per_s gpurun_out/${T}_hostapi_*.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1; rb=$?
echo "bench rc=$rb"; tail -c 1500 gpurun_out/${T}_bench.log
[ $rb -eq 0 ] || exit $rb
exit $rc
