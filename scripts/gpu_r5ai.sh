set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=3 bash scripts/ab_envs.sh r5aiab "grid||product" "nogrid|ORBX_TRACK_SKIP_GRID=1|product"
