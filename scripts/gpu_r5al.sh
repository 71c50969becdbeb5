set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_PROJ_A_THREADS=512 timeout -k 10 600 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_tracking.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5al_pytest.log 2>&1; rc=$?
echo "pytest (512) rc=$rc"; tail -2 gpurun_out/r5al_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh r5alab "a1024||product" "a512|ORBX_PROJ_A_THREADS=512|product" "a768|ORBX_PROJ_A_THREADS=768|product"
