# r6ze: the keyframe stream confined to k CUs (--kf-cus) against every CU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${ROUNDS:-2} bash scripts/ab_envs.sh ${TAG:-r6ze}ab "all||product" "kf128||product|--kf-cus 128" \
  "kf64||product|--kf-cus 64" "kf32||product|--kf-cus 32"
