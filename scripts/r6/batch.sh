# A/B of stereo frames per step (bench --batch), default schedule, side legs off; two rounds, alternating.
# usage: bash scripts/r6/batch.sh TAG "256 384 512"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r6batch}; BS=${2:-"256 384 512"}
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 30"
for r in 1 2; do for b in $BS; do
  timeout -k 10 300 python -u bench.py $B --batch $b > gpurun_out/${TAG}_b${b}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_b${b}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_b${b}_$r.log').read().strip().splitlines()[-1]); print('batch $b round $r', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d.get('stage_ms_per_step',{}).items()})"
done; done
