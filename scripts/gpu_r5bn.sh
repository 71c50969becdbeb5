# r5bn: with the quadtree of levels >= 1 on the stereo queue, the tracking searches on the keyframe queue instead
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5bnab "stereo||product" "kf|ORBX_BENCH_TRACK_STREAM=kf|product"
