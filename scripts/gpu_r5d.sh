set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r5d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rfs --timeout 300 --timeout-method thread -k "resize_pair or pyramid" \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=1 bash scripts/ab_envs.sh ${TAG}ab "base||product" "pk6|ORBX_RESIZE_PAIR=1|product" "pk4|ORBX_RESIZE_PAIR=1|build/pk4/liborbx.so" \
    "pk8|ORBX_RESIZE_PAIR=1|build/pk8/liborbx.so" "pk12|ORBX_RESIZE_PAIR=1|build/pk12/liborbx.so"
