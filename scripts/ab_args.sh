# A/B of bench arguments (no CPU / C3 / host-API legs): scripts/ab_args.sh "--diag-skip stereo" "" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 $a > gpurun_out/aa_$i.log 2>&1 || { echo "[$a] failed"; tail -3 gpurun_out/aa_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/aa_$i.log').read().strip().splitlines()[-1]); print('[$a]', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d.get('stage_ms_per_step', {}).items()})"
done
