# r5bl: quadtree of levels >= 1 on the side stream (ORBX_QT_OUT=2) against the output stream (default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_QT_OUT=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_ordering.py::test_canary_fires_when_an_edge_is_missing > gpurun_out/r5bl_pytest.log 2>&1 || { tail -30 gpurun_out/r5bl_pytest.log; exit 1; }
tail -1 gpurun_out/r5bl_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5blab "out||product" "side|ORBX_QT_OUT=2|product"
