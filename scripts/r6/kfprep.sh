# (ORBX_KF_PREP_THREADS, used by r6q below, was removed after the measurement: 1,024 threads fixed)
# r6p: k_kf_prep (a new keyframe's MapPoints + grid in one workgroup) -- its tests, then A/B against the two-launch form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6p}
timeout -k 10 500 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_fusion.py tests/test_gpu_tracking.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "split|ORBX_KF_PREP_SPLIT=1|product" "kf1024||product" "kf256|ORBX_KF_PREP_THREADS=256|product"
