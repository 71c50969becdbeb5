# r5cb: k_stereo_blk 128 right / 32 left keypoints per round (7.2 KB LDS) against 256 / 64 (product)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_LIB=build/sb128/liborbx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cb_pytest.log 2>&1 || { tail -30 gpurun_out/r5cb_pytest.log; exit 1; }
tail -1 gpurun_out/r5cb_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5cbab "s256||product" "s128||build/sb128/liborbx.so"
