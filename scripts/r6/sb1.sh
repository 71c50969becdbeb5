# r6b: k_describe_sb (blur at the BRIEF samples, ORBX_DESC_SB=1): extraction parity, then A/B against k_blur7 + k_describe_m
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6b}
ORBX_DESC_SB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_ordering.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_sb.log 2>&1; rc=$?
tail -30 gpurun_out/${T}_pytest_sb.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "base||product" "sb|ORBX_DESC_SB=1|product"
