# r5bt: keyframe stream at normal priority (and the stereo queue at high), combinations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=3 bash scripts/ab_envs.sh r5btab "base||product" "kf0|ORBX_KF_PRIORITY=0|product" "kf0stm1|ORBX_KF_PRIORITY=0 ORBX_STEREO_PRIORITY=-1|product" && \
AB_ARGS="--emulate-agents 8" ROUNDS=1 bash scripts/ab_envs.sh r5bt8 "base||product" "kf0|ORBX_KF_PRIORITY=0|product"
