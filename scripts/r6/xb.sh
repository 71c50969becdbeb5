# r6zl: the resize window column computed in the lane (no table load ahead of the window loads) -- the extraction
# tests, then A/B against the tree before (build/pre_xb)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6zl}
timeout -k 10 500 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} bash scripts/ab_envs.sh ${T}ab "before||$R/build/pre_xb/liborbx.so" "xb||product"
