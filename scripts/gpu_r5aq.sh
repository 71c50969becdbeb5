set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_tracking.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5aq_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5aq_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh r5aqab "fused||product" "two|ORBX_TRACK_TWO_LAUNCH=1|product"
