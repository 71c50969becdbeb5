# r6zm: the describe's keypoint position loaded beside the level counts (one round trip less before the window loads)
# -- the extraction tests (both describe forms), then A/B against the tree before (build/pre_xy)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6zm}
timeout -k 10 500 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} bash scripts/ab_envs.sh ${T}ab "before||$R/build/pre_xy/liborbx.so" "xy||product"
