# r6zc: k_kf_prep at 512 threads per workgroup (compile-time ORBX_KF_PREP_WG, build/kf512) against 1,024
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${ROUNDS:-3} bash scripts/ab_envs.sh ${TAG:-r6zc}ab "kf1024||product" "kf512||$R/build/kf512/liborbx.so"
