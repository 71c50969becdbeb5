# r6f: the keyframe all-gather straight into the ring slots (engine.exchange_view, commit in place): fusion tests, the
# world-2 gloo rehearsal, then the emulated-agent A/B (8 agents) against the round-5 gathered buffer + copy
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_multirank.py tests/test_multiagent.py -m gpu -x -q -rfs --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} AB_ARGS="--emulate-agents 8" bash scripts/ab_envs.sh ${T}emu "copy8||product|--exchange-copy" "ring8||product"
