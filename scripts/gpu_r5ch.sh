# r5ch: the assigning projection searches' candidate lists in global memory (ORBX_PROJ_GLIST=1; LDS ~70 KB per
# 1,024-thread workgroup instead of ~158 KB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_PROJ_GLIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_tracking.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ch_pytest.log 2>&1 || { tail -30 gpurun_out/r5ch_pytest.log; exit 1; }
tail -1 gpurun_out/r5ch_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5chab "lds||product" "gl|ORBX_PROJ_GLIST=1|product" "gl4|ORBX_PROJ_GLIST=1 ORBX_PROJ_LIST_MAX=4|product"
