# r5bu: the launch streams at high priority, with the keyframe stream at normal (new default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5buab "base||product" "mainm1|ORBX_MAIN_PRIORITY=-1|product" "kfm1|ORBX_KF_PRIORITY=-1|product"
