# A/B of one environment switch in one GPU call: bash scripts/ab_env_r4.sh TAG VAR "v1 v2 ..." [reps]
# (the bench's timed step only; every side block off)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; VAR=$2; VALS=$3; REPS=${4:-1}
for r in $(seq $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 \
        --alone-reps ${ALONE:-0} > gpurun_out/${T}_${v//\//_}_$r.log 2>&1 || exit $?
    echo "$VAR=$v rep $r $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${v//\//_}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_${v//\//_}_$r.log)"
    [ "${ALONE:-0}" != 0 ] && grep -o "\"stage_ms_alone\": {[^}]*}" gpurun_out/${T}_${v//\//_}_$r.log
  done
done
