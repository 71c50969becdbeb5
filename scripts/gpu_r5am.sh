set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5amab "base||product" "hwq8|ORBX_HW_QUEUES=8|product" "own8|ORBX_HW_QUEUES=8 ORBX_BENCH_TRACK_STREAM=own|product" "desc8|ORBX_HW_QUEUES=8 ORBX_BENCH_DESC_STREAM=2|product" "own4|ORBX_BENCH_TRACK_STREAM=own|product"
