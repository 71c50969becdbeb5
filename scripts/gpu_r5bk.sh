# r5bk: quadtree of levels >= 1 on the output stream by default -- full GPU suite, A/B against HEAD (launch stream)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bk_pytest.log 2>&1 || { tail -30 gpurun_out/r5bk_pytest.log; exit 1; }
tail -1 gpurun_out/r5bk_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5bkab "new||product" "base||build/base/liborbx.so" "old|ORBX_QT_OUT=0|product" && \
AB_ARGS="--config euroc" ROUNDS=1 bash scripts/ab_envs.sh r5bkeu "new||product" "old|ORBX_QT_OUT=0|product"
