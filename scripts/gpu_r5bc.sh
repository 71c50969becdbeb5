# r5bc: describe with one keypoint per wave (52 VGPRs, 5.9 KB LDS per workgroup) against two (64, 11.8 KB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_DESC_KPW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bc_pytest.log 2>&1 || { tail -30 gpurun_out/r5bc_pytest.log; exit 1; }
tail -1 gpurun_out/r5bc_pytest.log
ROUNDS=3 bash scripts/ab_envs.sh r5bcab "k2||product" "k1|ORBX_DESC_KPW=1|product"
