# r5bi: the Fuse search (non-assigning, 512 threads) staged in LDS (~44 KB per workgroup) or walking memory
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_PROJ_NA_STAGE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_tracking.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bi_pytest.log 2>&1 || { tail -30 gpurun_out/r5bi_pytest.log; exit 1; }
tail -1 gpurun_out/r5bi_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5biab "st||product" "mem|ORBX_PROJ_NA_STAGE=0|product"
