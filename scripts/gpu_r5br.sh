# r5br: FAST candidates double-buffered per call (call k + 1's FAST no longer waits for call k's quadtree on the
# output stream) -- GPU suite, A/B against HEAD and ORBX_CAND_SETS=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5br_pytest.log 2>&1 || { tail -30 gpurun_out/r5br_pytest.log; exit 1; }
tail -1 gpurun_out/r5br_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5brab "cs2||product" "base||build/base/liborbx.so" "cs1|ORBX_CAND_SETS=1|product"
