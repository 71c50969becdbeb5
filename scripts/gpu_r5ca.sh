# r5ca: k_stereo_blk with 256 right / 64 left keypoints staged per round (14.3 KB LDS per workgroup, was 28.7 KB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_stereo_refine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ca_pytest.log 2>&1 || { tail -30 gpurun_out/r5ca_pytest.log; exit 1; }
tail -1 gpurun_out/r5ca_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5caab "new||product" "base||build/base/liborbx.so"
