# (Record: the fused form was reverted after r7k; this script ran against that tree.)
# Stereo median rejection fused into k_stereo_sad_rows (last workgroup per pair) vs its own launch (ORBX_MEDIAN_SPLIT
# build): the stereo / tracking / smoke parity tests on the product library, then the A/B.  usage: bash scripts/r6/median.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r7med}
timeout -k 10 400 python -u -m pytest tests/test_stereo_refine.py tests/test_gpu_match.py tests/test_gpu_tracking.py tests/test_gpu_multirank.py \
    -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ORBX_LIB=build/msplit/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_stereo_refine.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/${T}_pytest_split.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest_split.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_envs.sh $T "fused||product" "split||build/msplit/liborbx.so"
