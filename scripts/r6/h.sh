# r6h: (1) C3 on the matrix cores (k_bf_mfma, ORBX_BF_MFMA=1): matcher tests in both forms, then the bench's C3 block
# (both forms, cross-checked); (2) the keyframe all-gather straight into the ring (engine.exchange_view): fusion tests,
# the world-2 gloo rehearsal, the emulated 8-agent A/B; (3) k_resize_tail (ORBX_RESIZE_TAIL=l): extraction parity at
# l = 4, A/B at l = 3, 4, 5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_match.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_match.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/micro/c3_only.py 2 > gpurun_out/${T}_c3.log 2>&1; rc=$?
cat gpurun_out/${T}_c3.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_multirank.py tests/test_multiagent.py -m gpu -x -q -rfs --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ORBX_RESIZE_TAIL=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_tail.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_tail.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 AB_ARGS="--emulate-agents 8" bash scripts/ab_envs.sh ${T}emu "copy8||product|--exchange-copy" "ring8||product" || exit 1
ROUNDS=2 bash scripts/ab_envs.sh ${T}tail "base||product" "tail3|ORBX_RESIZE_TAIL=3|product" "tail4|ORBX_RESIZE_TAIL=4|product" "tail5|ORBX_RESIZE_TAIL=5|product"
