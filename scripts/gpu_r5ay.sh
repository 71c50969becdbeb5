# r5ay: k_kfdb_pairwise over per-query vocabulary bitmaps in memory -- GPU suite (and the kfdb tests on the hash form), A/B at 8 and 1 agents
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ay_pytest.log 2>&1 || { tail -30 gpurun_out/r5ay_pytest.log; exit 1; }
tail -2 gpurun_out/r5ay_pytest.log
ORBX_KFDB_BITMAP=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_kfdb.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ay_pytest_hash.log 2>&1 || { tail -30 gpurun_out/r5ay_pytest_hash.log; exit 1; }
tail -1 gpurun_out/r5ay_pytest_hash.log
AB_ARGS="--emulate-agents 8" ROUNDS=2 bash scripts/ab_envs.sh r5ayab8 "gb||product" "hash|ORBX_KFDB_BITMAP=0|product" && \
ROUNDS=2 bash scripts/ab_envs.sh r5ayab1 "gb||product" "hash|ORBX_KFDB_BITMAP=0|product"
