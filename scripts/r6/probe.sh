# r6a: the k_describe_sb hardware probe (unaligned 32-bit LDS reads, i8 MFMA operand map, MFMA cycles), then the
# default bench once for this round's first figure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 60 build/mx_probe > gpurun_out/r6a_mx_probe.log 2>&1; rc=$?
cat gpurun_out/r6a_mx_probe.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=1 bash scripts/ab_envs.sh r6a "base||product"
