# Per-rank step under an N-agent keyframe load (bench.py --emulate-agents N, one GPU): how the keyframe path grows with N.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-emu}
for n in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --emulate-agents $n --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 \
      --alone-reps 0 > gpurun_out/${TAG}_n$n.log 2>&1 || { echo "n=$n failed"; tail -5 gpurun_out/${TAG}_n$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_n$n.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']
print('agents $n', d['value'], d['ms_per_step'], 'kf', s.get('keyframe_bow_fusion'), 'tri', s.get('keyframe_new_mappoints'), 'fuse', s.get('keyframe_fuse'), 'gate', d['fusion_gate_passed_per_step'], 'host', d['host_wall_split_ms_per_timed_step'])"
done
