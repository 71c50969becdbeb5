set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5aeab "inner2w5||build/inner2w5/liborbx.so" "bw5||build/bw5/liborbx.so" "bw4||build/bw4/liborbx.so" "in1w5||build/in1w5/liborbx.so" "in2w4||build/in2w4/liborbx.so" "base||product"
