# A/B of bench argument sets (default legs off): ARGS_LIST="|--inflight 2|--inflight 2 --batch 64" (| separated)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3ak}
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
IFS='|' read -ra LIST <<< "${ARGS_LIST}"
i=0
for a in "${LIST[@]}" "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py $B $a > gpurun_out/${TAG}_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_$i.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_$i.log').read().strip().splitlines()[-1]); print('[$a]', d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d.get('stage_ms_per_step',{}).items()})"
done
