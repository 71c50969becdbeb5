set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5aj_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5aj_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh r5ajab "ingrid||product" "launch|ORBX_TRACK_GRID_LAUNCH=1|product"
