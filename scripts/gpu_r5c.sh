set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r5c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfs --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=1 bash scripts/ab_envs.sh ${TAG}ab "base||product" "pk6|ORBX_RESIZE_PAIR=1|product" "pk4|ORBX_RESIZE_PAIR=1|build/pk4/liborbx.so" \
    "pk8|ORBX_RESIZE_PAIR=1|build/pk8/liborbx.so" "pk12|ORBX_RESIZE_PAIR=1|build/pk12/liborbx.so" "base2||product"
