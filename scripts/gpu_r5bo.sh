# r5bo: quadtree LDS key capacities re-swept with the levels >= 1 quadtree on the stereo queue
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_envs.sh r5boab "base||product" "k1_1k|ORBX_QT_KEYS1=1024|product" "k1_0|ORBX_QT_KEYS1=0|product" "k0_1k|ORBX_QT_KEYS0=1024|product" "k0_5k|ORBX_QT_KEYS0=5808|product"
