# A/B of environment settings on the default bench (no CPU / C3 / host-API legs): scripts/ab_env.sh "A=1" "A=0 B=2" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 > gpurun_out/ab_$i.log 2>&1 || { echo "[$cfg] failed"; tail -3 gpurun_out/ab_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); print('[$cfg]', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})"
done
