# r5bg: k_quadtree level-0 LDS key capacity sweep (default 5808 keys, 82 KB per workgroup)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5bgab "base||product" "k0_0|ORBX_QT_KEYS0=0|product" "k0_1k|ORBX_QT_KEYS0=1024|product" "k0_2k|ORBX_QT_KEYS0=2048|product" "k0_3k|ORBX_QT_KEYS0=3072|product" "k0_4k|ORBX_QT_KEYS0=4096|product"
