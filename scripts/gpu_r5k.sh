set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kfdb.py tests/test_gpu_kfdb_concurrency.py tests/test_gpu_fusion.py tests/test_gpu_cd.py tests/test_multiagent.py -m gpu -x -q -rfs --timeout 200 --timeout-method thread \
    > gpurun_out/r5k_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r5k_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_emu.sh r5k
