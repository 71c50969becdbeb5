# r5bh: k_quadtree level-0 keys capped at 3,072 (new default) against HEAD; levels >= 1 key capacity 1,024 / 512 (A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bh_pytest.log 2>&1 || { tail -30 gpurun_out/r5bh_pytest.log; exit 1; }
tail -1 gpurun_out/r5bh_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5bhab "new||product" "base||build/base/liborbx.so" "k1_1k|ORBX_QT_KEYS1=1024|product" "k1_512|ORBX_QT_KEYS1=512|product"
