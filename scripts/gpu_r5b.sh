set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r5b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_tracking.py tests/test_gpu_proj.py \
    tests/test_gpu_multirank.py -m gpu -x -q -rfs --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/ab_envs.sh ${TAG}ab "base||product" "sw36||build/sw36/liborbx.so" "pair|ORBX_RESIZE_PAIR=1|product" \
    "fsplit|ORBX_FUSE_SPLIT=1|product"
