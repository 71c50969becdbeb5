set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=3 bash scripts/ab_envs.sh r5sab "dsets2||product" "dsets1|ORBX_DESC_SETS=1|product"
