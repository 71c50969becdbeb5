set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=1 bash scripts/ab_envs.sh r5qab "base||product" "stop1||build/stop1/liborbx.so" "stop2||build/stop2/liborbx.so" "stop3||build/stop3/liborbx.so" "u8sc||build/u8sc/liborbx.so"
