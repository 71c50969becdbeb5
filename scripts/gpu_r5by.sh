# r5by: 8 hardware queues per process (GPU_MAX_HW_QUEUES via ORBX_HW_QUEUES) under the r5bk / r5bt schedule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5byab "base||product" "hwq8|ORBX_HW_QUEUES=8|product" "hwq8kfm1|ORBX_HW_QUEUES=8 ORBX_KF_PRIORITY=-1|product"
