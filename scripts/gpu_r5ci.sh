# r5ci: the blur of levels 1..n-1 on the output (stereo) queue ahead of the quadtree (ORBX_BLUR_OUT=1) instead of the
# side stream
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_BLUR_OUT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_ordering.py::test_canary_fires_when_an_edge_is_missing > gpurun_out/r5ci_pytest.log 2>&1 || { tail -30 gpurun_out/r5ci_pytest.log; exit 1; }
tail -1 gpurun_out/r5ci_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5ciab "side||product" "out|ORBX_BLUR_OUT=1|product"
