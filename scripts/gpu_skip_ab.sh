# Critical-path probe (diagnostics): the default step vs the step without the keyframe path / without stereo + keyframes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3aj}
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
for v in ${FORMS:-none keyframes stereo none keyframes stereo}; do
  A=""; [ $v != none ] && A="--diag-skip $v"
  timeout -k 10 300 python -u bench.py $B $A > gpurun_out/${TAG}_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_$v.log').read().strip().splitlines()[-1]); print('skip $v', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d.get('stage_ms_per_step',{}).items()})"
done
