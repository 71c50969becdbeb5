# r5bs: stream priorities re-checked under the r5bk schedule (env only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5bsab "base||product" "sp0|ORBX_SIDE_PRIORITY=0|product" "stm1|ORBX_STEREO_PRIORITY=-1|product" "kf0|ORBX_KF_PRIORITY=0|product" "na1024|ORBX_PROJ_NA_THREADS=1024|product"
