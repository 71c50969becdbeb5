# Ordering diagnostics (round 3): HIP stream-ordering micro, the ordering tests, the configure-upload race A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r3}
timeout -k 5 60 scripts/micro/stream_order > gpurun_out/${TAG}_stream_order.log 2>&1; echo "micro rc=$?"; cat gpurun_out/${TAG}_stream_order.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ordering.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_ordering_pytest.log 2>&1; rc=$?; echo "ordering tests rc=$rc"; tail -15 gpurun_out/${TAG}_ordering_pytest.log
[ $rc -eq 0 ] || exit $rc
ORBX_LIB=build/legacy/liborbx.so timeout -k 10 240 python -u scripts/diag/upload_race.py 0.4 41 2 > gpurun_out/${TAG}_upload_race_legacy.log 2>&1 || exit $?
tail -8 gpurun_out/${TAG}_upload_race_legacy.log
timeout -k 10 240 python -u scripts/diag/upload_race.py 0.4 41 2 > gpurun_out/${TAG}_upload_race_fixed.log 2>&1 || exit $?
tail -4 gpurun_out/${TAG}_upload_race_fixed.log
