set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_proj.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5ah_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5ah_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh r5ahab "found||product" "torch|ORBX_TRACK_TORCH_FOUND=1|product"
