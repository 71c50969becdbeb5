# A/B of bench argument sets in one GPU call: bash scripts/ab_args_r4.sh TAG "args1" "args2" ... (timed step only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
for rep in ${REPS:-1}; do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 \
        --alone-reps 0 $a > gpurun_out/${T}_${i}_$rep.log 2>&1 || exit $?
    echo "[$a] rep $rep $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${i}_$rep.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_${i}_$rep.log)"
  done
done
