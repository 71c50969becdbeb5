set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for a in ${ABL:-1 2 3 0}; do
  ORBX_FAST_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/abl_$a.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$a.log').read().strip().splitlines()[-1]); print('ablate $a', d['stage_ms_per_step'])"
done
