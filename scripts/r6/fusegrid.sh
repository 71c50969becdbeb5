# r6e: k_describe_sb parity + A/B (aligned reads, shared loads); the Fuse search building the new keyframes' grids
# (no k_grid_count launch) -- its tests, then A/B against ORBX_FUSE_GRID_LAUNCH=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6e}
ORBX_DESC_SB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_sb.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_sb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_proj.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_fuse.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_fuse.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "base|ORBX_FUSE_GRID_LAUNCH=1|product" "fgrid||product" "sb|ORBX_DESC_SB=1|product"
