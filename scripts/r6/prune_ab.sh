# r6zb: the pruned tree (k_stereo / k_stereo_sad and 17 knobs removed) against the tree before it (b1fd4c1, built into
# build/r6w_tree/) on one box: the default path should not move
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${ROUNDS:-3} bash scripts/ab_envs.sh ${TAG:-r6zb}ab "before||$R/build/r6w_tree/liborbx.so" "pruned||product"
