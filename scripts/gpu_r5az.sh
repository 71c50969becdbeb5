# r5az: k_kfdb_score workgroups past the query's candidates leave before staging; k_grid_count at 256 threads (A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kfdb.py tests/test_gpu_fusion.py tests/test_gpu_kfdb_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5az_pytest.log 2>&1 || { tail -30 gpurun_out/r5az_pytest.log; exit 1; }
tail -1 gpurun_out/r5az_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5azab1 "new||product" "base||build/base/liborbx.so" "gt256|ORBX_GRID_THREADS=256|product" && \
AB_ARGS="--emulate-agents 8" ROUNDS=2 bash scripts/ab_envs.sh r5azab8 "new||product" "base||build/base/liborbx.so"
