# A/B of library builds on the default bench (no CPU / C3 / host-API legs): scripts/ab_lib.sh product build/x/liborbx.so ...
# ("product" = the in-tree liborbx.so).  Extra env for every run: AB_ENV="A=1 B=2".
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
i=0
for lib in "$@"; do
  i=$((i+1))
  L=""; [ "$lib" != product ] && L="ORBX_LIB=$lib"
  env $L $AB_ENV timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 > gpurun_out/al_$i.log 2>&1 || { echo "[$lib] failed"; tail -3 gpurun_out/al_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/al_$i.log').read().strip().splitlines()[-1]); print('[$lib]', d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})"
done
