set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do for e in "ORBX_KFDB_PAIRWISE_MAX=2048" "ORBX_KFDB_PAIRWISE_MAX=0"; do
  env $e timeout -k 10 200 python -u bench.py --emulate-agents 8 --cpu-seconds 0 --no-c3 --host-api-frames 0 --no-cd --host-fed-steps 0 \
      --alone-reps 0 > gpurun_out/r5m.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/r5m.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r5m.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']
print('$e', d['value'], d['ms_per_step'], 'kf', s.get('keyframe_bow_fusion'), 'gate', d['fusion_gate_passed_per_step'])"
done; done
