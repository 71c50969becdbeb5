# r5cc: k_stereo_sad_rows' row shares as u16 in LDS (6.2 KB per workgroup, was 11.4 KB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_stereo_refine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cc_pytest.log 2>&1 || { tail -30 gpurun_out/r5cc_pytest.log; exit 1; }
tail -1 gpurun_out/r5cc_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5ccab "new||product" "base||build/base/liborbx.so"
