set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5adab "base||product" "inner1||build/inner1/liborbx.so" "inner2||build/inner2/liborbx.so" "inner2w5||build/inner2w5/liborbx.so"
