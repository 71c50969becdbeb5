# r5bj: DistributeOctTree of levels 1..n-1 on the output stream (ORBX_QT_OUT=1): the launch stream goes on to the next
# call's resize chain right after FAST
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_QT_OUT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py tests/test_gpu_concurrency.py tests/test_gpu_tracking.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_ordering.py::test_canary_fires_when_an_edge_is_missing > gpurun_out/r5bj_pytest.log 2>&1 || { tail -30 gpurun_out/r5bj_pytest.log; exit 1; }
tail -1 gpurun_out/r5bj_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5bjab "base||product" "qto|ORBX_QT_OUT=1|product"
