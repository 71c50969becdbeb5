set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kfdb_concurrency.py tests/test_gpu_kfdb.py tests/test_gpu_concurrency.py tests/test_gpu_match.py tests/test_gpu_proj.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/r3d_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tsan_gpu.sh 10; rc=$?; cp gpurun_out/tsan.log gpurun_out/r3d_tsan.log; exit $rc
