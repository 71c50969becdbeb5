# r5ck: the Fuse search (non-assigning) at 256 / 384 threads under the current schedule (env only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5ckab "base||product" "na256|ORBX_PROJ_NA_THREADS=256|product" "na384|ORBX_PROJ_NA_THREADS=384|product"
