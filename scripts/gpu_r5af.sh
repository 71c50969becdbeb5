set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5af_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5af_pytest.log
[ $rc -eq 0 ] || exit $rc
ORBX_BLUR_WGX=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5af_pytest_wgx64.log 2>&1; rc=$?
echo "pytest wgx64 rc=$rc"; tail -1 gpurun_out/r5af_pytest_wgx64.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/ab_envs.sh r5afab "none||product" "wgx128|ORBX_BLUR_WGX=128|product" "wgx96|ORBX_BLUR_WGX=96|product" "wgx64|ORBX_BLUR_WGX=64|product"
