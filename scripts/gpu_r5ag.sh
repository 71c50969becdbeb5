set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5agab "base||product" "desc96||build/desc96/liborbx.so" "desc80||build/desc80/liborbx.so" "rs96||build/rs96/liborbx.so" "rs128||build/rs128/liborbx.so" "bl128||build/bl128/liborbx.so"
