set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=3 bash scripts/ab_envs.sh r5tab "base||product" "main_hi|ORBX_MAIN_PRIORITY=-1|product"
