# r6c: k_describe_sb with 4-byte-aligned sample reads: extraction parity, then A/B against k_blur7 + k_describe_m
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6c}
ORBX_DESC_SB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_sb.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest_sb.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "base||product" "sb|ORBX_DESC_SB=1|product"
