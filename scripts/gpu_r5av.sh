# r5av: k_blur7 band height A/B (32 = product, 24 / 48 / 16 rows per tile)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5avab "bb32||product" "bb24||build/bb24/liborbx.so" "bb48||build/bb48/liborbx.so" "bb16||build/bb16/liborbx.so"
