# r6zf: the keyframe stream confined to k CUs at 1 and 8 emulated agents
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${TAG:-r6zf}ab "all||product" "kf64||product|--kf-cus 64" \
  "kf16||product|--kf-cus 16" "all8||product|--emulate-agents 8" "kf64_8||product|--kf-cus 64 --emulate-agents 8" \
  "kf32_8||product|--kf-cus 32 --emulate-agents 8"
