# r6u: the keyframe database's word map -- its tests, then A/B against the pairwise form at 1 and 8 emulated agents
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6u}
timeout -k 10 500 python -u -m pytest tests/test_gpu_kfdb.py tests/test_gpu_cd.py tests/test_gpu_kfdb_concurrency.py tests/test_gpu_fusion.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "pw1|ORBX_KFDB_WORDMAP=0|product" "wm1||product" \
  "pw8|ORBX_KFDB_WORDMAP=0|product|--emulate-agents 8" "wm8||product|--emulate-agents 8"
