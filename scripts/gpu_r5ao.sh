set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5ao_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5ao_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/ab_envs.sh r5aoab "dc16||product" "dc16w7||build/dc16w7/liborbx.so" "dc8||build/dc8/liborbx.so"
