# Round 4, GPU call d: the tracking / Fuse tests, then a kernel trace of the bench's steps (per-kernel times of the
# tracking and Fuse stages).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_proj.py -m gpu -x -q -rf --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
O=gpurun_out/${T}_kt; rm -rf $O; mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O" -o run -- python3 "$R/bench.py" \
    --steps 20 --warmup 5 --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --alone-reps 0 \
    > $O/kt.log 2>&1; rb=$?
echo "kt rc=$rb"; tail -c 600 $O/kt.log
exit $rc
