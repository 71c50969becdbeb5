# A/B of frames per step (bench --batch): default schedule, no CPU / C3 / host-API / CD / host-fed legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3ag}
B="--cpu-seconds 0 --host-api-frames 0 --no-c3 --no-cd --host-fed-steps 0 --steps 20"
for b in ${BATCHES:-128 192 256 128 192 256}; do
  timeout -k 10 300 python -u bench.py $B --batch $b > gpurun_out/${TAG}_b$b.log 2>&1 || { tail -5 gpurun_out/${TAG}_b$b.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_b$b.log').read().strip().splitlines()[-1]); print('batch $b', d['value'], d['ms_per_step'])"
done
