# r6j: C3 matcher tests in both forms, then the bench's C3 block twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_match.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_match.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/micro/c3_only.py 2 > gpurun_out/${T}_c3.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_c3.log; [ $rc -eq 0 ] || exit $rc
