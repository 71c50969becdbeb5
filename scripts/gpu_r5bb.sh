# r5bb: list slots per query of the assigning projection searches (LDS per 1024-thread workgroup: ~158 KB at the
# default, as many slots as 160 KB holds up to 16) -- fewer slots leave LDS to FAST beside them
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_PROJ_LIST_MAX=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_proj.py tests/test_gpu_tracking.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bb_pytest.log 2>&1 || { tail -30 gpurun_out/r5bb_pytest.log; exit 1; }
tail -1 gpurun_out/r5bb_pytest.log
ROUNDS=2 bash scripts/ab_envs.sh r5bbab "l16||product" "l0|ORBX_PROJ_LIST_MAX=0|product" "l2|ORBX_PROJ_LIST_MAX=2|product" "l4|ORBX_PROJ_LIST_MAX=4|product" "l8|ORBX_PROJ_LIST_MAX=8|product"
