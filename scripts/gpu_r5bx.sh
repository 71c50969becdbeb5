# r5bx: earlier knobs re-checked under the r5bk / r5bt schedule (env only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5bxab "base||product" "rpair|ORBX_RESIZE_PAIR=1|product" "gt512|ORBX_GRID_THREADS=512|product" "at768|ORBX_PROJ_A_THREADS=768|product" "ds1|ORBX_DESC_SETS=1|product"
