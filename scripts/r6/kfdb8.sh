# r6t: the keyframe database's two strategies at 8 emulated agents (pairwise bitmap vs inverted file), and 1 agent
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6t}
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${T}ab "one||product" "pw8||product|--emulate-agents 8" \
  "if8|ORBX_KFDB_PAIRWISE_MAX=0|product|--emulate-agents 8"
