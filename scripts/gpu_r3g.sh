set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ordering.py tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r3g_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3g_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms_per_step": {[^}]*}' gpurun_out/r3g_bench.log | head -4; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_r3.sh r3g_prof
