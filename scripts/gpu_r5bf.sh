# r5bf: k_quadtree's LDS-resident keys (level 0: ~82 KB per workgroup, levels >= 1: ~53 KB) against fewer LDS keys
# (the rest in the HBM scratch): LDS beside FAST
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ORBX_QT_VERBOSE=1 timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 --alone-reps 0 > gpurun_out/r5bf_verbose.log 2>&1 || { tail -5 gpurun_out/r5bf_verbose.log; exit 1; }
grep "k_quadtree LDS" gpurun_out/r5bf_verbose.log | head -2
ROUNDS=2 bash scripts/ab_envs.sh r5bfab "base||product" "k1z|ORBX_QT_KEYS1=0|product" "k0h|ORBX_QT_KEYS0=2048|product" "both|ORBX_QT_KEYS0=2048 ORBX_QT_KEYS1=0|product"
