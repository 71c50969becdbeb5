# A/B of environment sets in one GPU call: bash scripts/ab_envs_r4.sh TAG "VAR=v VAR2=w" ... (timed step only; "-" = none)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
for rep in ${REPS:-1}; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e="ORBX_NONE=1"
    env $e timeout -k 10 300 python -u bench.py --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 \
        --alone-reps 0 ${ARGS:-} > gpurun_out/${T}_${i}_$rep.log 2>&1 || exit $?
    echo "[$e] rep $rep $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${i}_$rep.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_${i}_$rep.log)"
  done
done
