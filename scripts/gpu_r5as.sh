set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_kfdb.py tests/test_gpu_kfdb_concurrency.py tests/test_gpu_fusion.py tests/test_gpu_cd.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5as_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5as_pytest.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--emulate-agents 8" ROUNDS=2 bash scripts/ab_envs.sh r5asab8 "new||product" "bw1|ORBX_BOW_WAVES=1|product" "base||build/base/liborbx.so"
ROUNDS=2 bash scripts/ab_envs.sh r5asab1 "new||product" "base||build/base/liborbx.so"
