# r5au: FAST second pass from the minThFAST masks kept by the first pass (pad words) -- GPU suite, then A/B vs HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5au_pytest.log 2>&1 || { tail -30 gpurun_out/r5au_pytest.log; exit 1; }
tail -3 gpurun_out/r5au_pytest.log
ROUNDS=3 bash scripts/ab_envs.sh r5auab "keep2||product" "base||build/base/liborbx.so"
