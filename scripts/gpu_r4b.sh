# Round 4, GPU call b: the matcher / KFDB stream-contract tests, the default bench, then the profile of the timed bench
# command (scripts/prof_r4.sh).  Each GPU step has its own time limit; any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kfdb_concurrency.py tests/test_gpu_concurrency.py tests/test_gpu_match.py \
    tests/test_gpu_kfdb.py tests/test_gpu_teardown.py tests/test_gpu_fusion.py -m gpu -x -q -rf --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -c 600 gpurun_out/${T}_bench.log
timeout -k 10 1000 bash scripts/prof_r4.sh ${T}_prof || exit 1
