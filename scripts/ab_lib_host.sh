# A/B of library builds with the host split of the timed steps: scripts/ab_lib_host.sh product build/x/liborbx.so ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
i=0
for lib in "$@"; do
  i=$((i+1))
  L=""; [ "$lib" != product ] && L="ORBX_LIB=$lib"
  env $L $AB_ENV timeout -k 10 200 python bench.py --cpu-seconds 0 --no-c3 --host-api-frames 0 $AB_ARGS > gpurun_out/ah_$i.log 2>&1 || { echo "[$lib] failed"; tail -3 gpurun_out/ah_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ah_$i.log').read().strip().splitlines()[-1]); print('[$lib]', d['value'], d['ms_per_step'], d['host_wall_ms_per_timed_step'], d['host_wall_split_ms_per_timed_step'], round(d['stage_ms_per_step']['keyframe_bow_fusion'], 3))"
done
