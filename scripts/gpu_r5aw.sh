# r5aw: keyframe-database strategy at 8 emulated agents (1,224 ring slots): pairwise intersection vs inverted file
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_ARGS="--emulate-agents 8" ROUNDS=2 bash scripts/ab_envs.sh r5awab8 "pw||product" "if|ORBX_KFDB_PAIRWISE_MAX=0|product"
