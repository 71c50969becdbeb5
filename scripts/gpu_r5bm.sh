# r5bm: DistributeOctTree of every level in one launch on the output stream (ORBX_QT_OUT=3) against levels 1..n-1 only
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_QT_OUT=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_ordering.py::test_canary_fires_when_an_edge_is_missing > gpurun_out/r5bm_pytest.log 2>&1 || { tail -30 gpurun_out/r5bm_pytest.log; exit 1; }
tail -1 gpurun_out/r5bm_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5bmab "out||product" "all|ORBX_QT_OUT=3|product"
