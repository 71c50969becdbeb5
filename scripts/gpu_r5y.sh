set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/diag/brief_diff.py 21 0 1 > gpurun_out/r5y_diff.log 2>&1; echo "diff rc=$?"; cat gpurun_out/r5y_diff.log | tail -30
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5y_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5y_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh r5yab "new||product" "base||build/base/liborbx.so"
